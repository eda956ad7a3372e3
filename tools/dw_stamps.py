"""GPU, variant library (tools/variants/lg_stamps.h): lg_decide_write's phases on C5's frame (stamps 0, 13, 14, 15),
medians over frames.  usage: CONES_GPU_LIB=lib_variants/lgst/libcones_gpu.so python tools/dw_stamps.py"""
import os, sys, statistics
import numpy as np
sys.path.insert(0, os.getcwd())
import cones_perception_amd as cp
from cones_perception_amd import _abi
import torch
raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
d = torch.from_numpy(raw).cuda()
eng = cp.BatchEngine(cp.load_params("simulation"))
rows = []
for it in range(60):
    eng.run(d.data_ptr(), 1, raw.shape[1] // 16, 16)
    torch.cuda.synchronize()
    st = np.zeros(64, np.uint64)
    _abi.check(_abi.lib().cg_debug_large_buffer(eng.handle, 4, st.ctypes.data, 512))
    if it >= 10:
        rows.append(st.astype(np.int64))
a = np.array(rows)
med = lambda x: float(np.median(x)) / 100.0
print("decide_write (ticket-0 block / last block), us from the block-0 start:")
print("  fold + thresholds", med(a[:, 13] - a[:, 0]))
print("  pass 2 + loads + scan + look-back + bounds", med(a[:, 14] - a[:, 13]))
print("  -> last block's fold done", med(a[:, 15] - a[:, 14]))
print("  last fold done -> pcl_index block 1 start", med(a[:, 58] - a[:, 15]))
print("  pcl_index start -> level 0 first stamp", med(a[:, 16] - a[:, 58]))
