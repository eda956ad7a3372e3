"""GPU, variant library (tools/variants/lg_stamps.h): lg_cluster_tail's phase times on C5's frame,
median over frames. usage: CONES_GPU_LIB=lib_variants/lgst/libcones_gpu.so python tools/lg_stamps.py"""
import ctypes as C
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cones_perception_amd as cp  # noqa: E402
from cones_perception_amd import _abi  # noqa: E402
import torch  # noqa: E402

raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
d = torch.from_numpy(raw).cuda()
eng = cp.BatchEngine(cp.load_params("simulation"))
names = ["start", "parents", "roots", "sizes", "filter", "order", "offsets", "labels", "csr", "xy", "centroids",
         "offs+header", "end"]
rows = []
for it in range(40):
    eng.run(d.data_ptr(), 1, raw.shape[1] // 16, 16)
    torch.cuda.synchronize()
    st = np.zeros(66, np.uint64)
    _abi.check(_abi.lib().cg_debug_large_buffer(eng.handle, 4, st.ctypes.data, 528))
    if it >= 5:
        rows.append(st.astype(np.int64))
t = np.array(rows)
print("lg_cluster_tail phases, us (median of %d frames):" % len(rows))
for i in range(2, 13):
    print(f"  {names[i - 1]:12s} {statistics.median((t[:, i] - t[:, i - 1]) / 100.0):7.2f}")
print(f"  total        {statistics.median((t[:, 12] - t[:, 1]) / 100.0):7.2f}")
print("lg_decide_write, workgroup 0 (fold of the front's keys + thresholds, pass 2 + survivor loads + "
      "look-back + bounds), then to the last arrival's fold end, us:")
for nm, a0, a1 in (("fold+thr", 0, 13), ("pass2..bounds", 13, 14), ("to last fold end", 14, 15), ("total", 0, 15)):
    print(f"  {nm:18s} {statistics.median((t[:, a1] - t[:, a0]) / 100.0):7.2f}")
if (t[:, 64] > t[:, 8]).all():   # the CSR's three parts (stamps 64, 65)
    for nm, a0, a1 in (("csr counts", 8, 64), ("csr starts", 64, 65), ("csr place", 65, 9)):
        print(f"  {nm:12s} {statistics.median((t[:, a1] - t[:, a0]) / 100.0):7.2f}")
# lg_pq_level, workgroup 0: split phase, wait for the range, swaps; gap from the previous level
allr = []
for it in range(20):
    eng.run(d.data_ptr(), 1, raw.shape[1] // 16, 16)
    torch.cuda.synchronize()
    st = np.zeros(64, np.uint64)
    _abi.check(_abi.lib().cg_debug_large_buffer(eng.handle, 4, st.ctypes.data, 512))
    allr.append(st.astype(np.int64))
a = np.array(allr[5:])
print("lg_pq_level, the workgroup holding tile 0, us: tiles+ticket -> look-back -> lists stored -> count added -> "
      "range complete -> swaps done; then to the next level's same point")
for lv in range(7):
    b = 16 + 6 * lv
    st_ = [a[:, b + i] for i in range(6)]
    nxt = a[:, b + 6] if lv < 6 else st_[5]
    med = lambda x: float(np.median(x)) / 100.0
    print(f"  level {lv}: lookback {med(st_[1] - st_[0]):6.2f}  lists {med(st_[2] - st_[1]):6.2f}  "
          f"count {med(st_[3] - st_[2]):6.2f}  wait {med(st_[4] - st_[3]):6.2f}  swaps {med(st_[5] - st_[4]):6.2f}  "
          f"to next {med(nxt - st_[5]):6.2f}")
print("lg_pcl_index (workgroup 1 / tile 1), us: grid setup, cstart zero + ticket, keys, look-back scan, emit + done")
for nm, i0, i1 in (("setup", 58, 59), ("zero+ticket", 59, 60), ("keys", 60, 61), ("scan", 61, 62), ("emit+done", 62, 63)):
    print(f"  {nm:12s} {float(np.median(a[:, i1] - a[:, i0])) / 100.0:7.2f}")
