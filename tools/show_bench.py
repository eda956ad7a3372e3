"""Summarise a bench output file (default gpurun_out/bench.log): the value line with its
sustained pass, C5 and C2 legs, and any phase stamps."""
import json
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.log"
for line in open(path):
    if line.startswith("{"):
        d = json.loads(line)
        r = d.get("roofline") or {}
        print("VALUE %.4g frames/s  %.4f ms/step  aggregate_frac %s  span_frac %s" % (
            d["value"], d["ms_per_step"], r.get("aggregate_frac"), r.get("frac")))
        s = d.get("sustained")
        if s and "value" in s:
            print("SUSTAINED %d steps %.4g frames/s aggregate %.3f span %.4f ms drift %+.3f overlap %+.3f pace %+.3f: %s" % (
                s["steps"], s["value"], s["aggregate_frac"], s["span_ms_mean"], s["span_drift_last_vs_first"],
                s["overlap_growth_last_vs_first"], s["step_time_change_last_vs_first"], s["finding"]))
        c5 = d.get("c5_single_gpu")
        if c5:
            print("C5", {k: c5.get(k) for k in ("ms_per_frame", "point_order_ms_per_frame", "error")})
        sf = d.get("single_frame")
        if sf:
            c = sf.get("cpp_node") or {}
            print("C2 python %.4f ms (p50 %s), cpp %s (p50 %s, p90 %s)" % (
                sf.get("latency_ms", float("nan")), sf.get("latency_p50_ms"), c.get("latency_ms"),
                c.get("latency_p50_ms"), c.get("latency_p90_ms")))
        if "ranks" in d:
            print("RANKS", d["ranks"])
        if "c5_tiled" in d:
            print("C5 TILED", json.dumps(d["c5_tiled"])[:600])
    elif line.startswith("STAMPS"):
        d = json.loads(line[7:])
        print(d.pop("tag"), json.dumps(d))
