"""Per-frame busy time, launch count and inter-launch gaps of the C5 large path, from the
rocprofv3 kernel trace tools/c5_kernels.sh writes (gpurun_out/c5k_<lib>/run_kernel_trace.csv).
usage: python tools/c5_gaps.py [trace.csv]"""
import collections
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c5k_default/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void lg_front")]
gaps, busy_k, per = collections.Counter(), collections.Counter(), []
for a, b in zip(starts[10:-1], starts[11:]):   # skip the first frames (warm-up)
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    per.append((t1 - t0, sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg), len(seg)))
    for x, y in zip(seg, seg[1:] + [rows[b]]):
        name = x["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        gaps[name] += int(y["Start_Timestamp"]) - int(x["End_Timestamp"])
        busy_k[name] += int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
n = len(per)
print(f"{n} frames (under the profiler): {sum(p[0] for p in per) / n / 1e3:.1f} us per frame, "
      f"{sum(p[1] for p in per) / n / 1e3:.1f} us of kernels, {sum(p[2] for p in per) / n:.1f} launches")
print(f"{'kernel':50s} {'busy us':>8s} {'gap after us':>13s}")
for k, v in busy_k.most_common():
    print(f"{k:50s} {v / n / 1e3:8.1f} {gaps[k] / n / 1e3:13.1f}")
