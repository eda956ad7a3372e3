"""Per-launch durations of the C5 large path in stream order (medians over the frames with the
most common launch sequence), from the rocprofv3 kernel trace tools/c5_kernels.sh writes.
usage: python tools/c5_launches.py [trace.csv]"""
import collections
import csv
import statistics
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c5k_default/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void lg_front")]
frames = [rows[a:b] for a, b in zip(starts[10:-1], starts[11:])]
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "")[:46]
seqs = collections.Counter(tuple(name(r) for r in f) for f in frames)
common, cnt = seqs.most_common(1)[0]
sel = [f for f in frames if tuple(name(r) for r in f) == common]
print(f"# C5 1M-point frame, PCL order: per-launch durations in stream order, medians over the {len(sel)} frames "
      f"with the common {len(common)}-launch sequence ({len(frames)} frames traced)")
print(f"{'#':>3s} {'kernel':46s} {'us':>8s} {'gap after us':>13s}")
tot = 0.0
for i, k in enumerate(common):
    d = statistics.median((int(f[i]["End_Timestamp"]) - int(f[i]["Start_Timestamp"])) / 1e3 for f in sel)
    g = statistics.median(((int(f[i + 1]["Start_Timestamp"]) if i + 1 < len(f) else int(f[i]["End_Timestamp"]))
                           - int(f[i]["End_Timestamp"])) / 1e3 for f in sel)
    tot += d
    print(f"{i:3d} {k:46s} {d:8.2f} {g:13.2f}")
span = statistics.median((int(f[-1]["End_Timestamp"]) - int(f[0]["Start_Timestamp"])) / 1e3 for f in sel)
print(f"sum of kernel medians: {tot:.1f} us over {len(common)} launches; first start to last end: {span:.1f} us")
