"""Summarise gpurun_out/bench.log: value line and phase stamps."""
import json
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.log"
for line in open(path):
    if line.startswith("{"):
        d = json.loads(line)
        print("VALUE %.4g frames/s  %.4f ms/step  aggregate_frac %.3f" % (
            d["value"], d["ms_per_step"], d["roofline"]["aggregate_frac"]))
    elif line.startswith("STAMPS"):
        d = json.loads(line[7:])
        print(d.pop("tag"), json.dumps(d))
