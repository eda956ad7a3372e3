"""Per-frame kernel time of the C5 large path from a rocprofv3 --stats csv:
    python tools/c5_stats.py gpurun_out/c5/run_kernel_stats.csv [frames]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 23
tot = 0.0
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    t = float(r["TotalDurationNs"]) / frames / 1e3
    tot += t
    print(f"{r['Name'][:58]:58s} {int(r['Calls']) / frames:5.1f}/frame {t:7.2f} us/frame")
print(f"total {tot:.1f} us of kernel time per frame")
