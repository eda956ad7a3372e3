"""GPU diagnostic: phase stamps of the C2 split single-frame launch (one 64k-point frame through
ConePipeline.cloud_handler). Per chunk workgroup: start (0), chunk published (27), chunk copied
to the device (28), pass 1 done and minima published (29), every chunk's minima merged (30), the
last workgroup past the survivors' count (31); its tail phases (1-20) in its own slot.
Times in us from the launch's first workgroup start, medians over the calls."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cones_perception_amd as cp  # noqa: E402
from cones_perception_amd import _abi  # noqa: E402

params = cp.load_params("simulation")
pipe = cp.ConePipeline(params)
msg = cp.frame_cloud(cp.synth_frames(1, first_frame=0, rings=64, cols=1024)[0])
lib = _abi.lib()
for _ in range(20):
    pipe.cloud_handler(msg)
_abi.check(lib.cg_debug_stamps(pipe.handle, 1))
calls = int(sys.argv[1]) if len(sys.argv) > 1 else 100
buf = np.zeros((16, 32), np.uint64)
rows = []
for _ in range(calls):
    pipe.cloud_handler(msg)
    _abi.check(lib.cg_debug_stamps_fetch(pipe.handle, buf.ctypes.data, 16))
    t = buf.astype(np.int64)
    t0 = t[t[:, 0] > 0, 0].min()
    rows.append(np.where(t > 0, (t - t0) / 100.0, np.nan))
a = np.nanmedian(np.stack(rows), axis=0)
names = {0: "start", 27: "published", 28: "copied", 29: "pass1 done", 30: "all arrived", 31: "last wg"}
print("chunk " + " ".join(f"{names[p]:>11s}" for p in (0, 27, 28, 29, 30, 31)))
for c in range(16):
    print(f"{c:5d} " + " ".join(f"{a[c, p]:11.2f}" for p in (0, 27, 28, 29, 30, 31)))
last = np.stack(rows)
lw = [int(np.nanargmax(np.nan_to_num(r[:, 20], nan=-1))) for r in rows]
tail = np.nanmedian(np.stack([r[w] for r, w in zip(rows, lw)]), axis=0)
print("last workgroup (median over calls):", {p: round(float(tail[p]), 2) for p in range(32) if not np.isnan(tail[p])})
