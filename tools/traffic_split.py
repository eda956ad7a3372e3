"""Per-frame HBM traffic of cg_frame_kernel (FETCH_SIZE x2, the gfx950 correction for wide
streaming reads, MI355X_MICROARCH.md; WRITE_SIZE as reported) for the default library and the
stop-after-phase variants, from the rocprofv3 CSVs tools/r5_traffic.sh writes."""
import csv
import glob
import json
import os
import statistics
import sys

O = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/traffic"
KERNEL = "cg_frame_kernel<128, 1, 0>("
F = 256


def med(lib, counter):
    got = glob.glob(os.path.join(O, f"{lib}_{counter}", "**", "run_counter_collection.csv"), recursive=True)
    per = {}
    for row in csv.DictReader(open(got[0])):
        if KERNEL in row["Kernel_Name"] and row["Counter_Name"] == counter:
            per[row["Dispatch_Id"]] = per.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return statistics.median(per.values()) * 1024 / F   # KB per dispatch -> bytes per frame


out = {}
for lib in ("stop1", "stop1aux0", "stop2", "stop3", "default", "aux0"):
    try:
        f, w = med(lib, "FETCH_SIZE"), med(lib, "WRITE_SIZE")
    except (IndexError, ValueError):
        continue
    out[lib] = {"fetch_x2_bytes_per_frame": 2 * f, "write_bytes_per_frame": w, "hbm_bytes_per_frame": 2 * f + w}
print(json.dumps(out, indent=1))
