"""Diagnostic: repeat the C5 frame through the large path and report any run-to-run
difference of K or of the per-sector minimum keys (meta words)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cones_perception_amd as cp  # noqa: E402
from cones_perception_amd import _abi  # noqa: E402

params = cp.load_params("simulation")
raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
msg = cp.frame_cloud(raw[0])
for name, obj in (("ground", cp.GroundRemover(params)), ("pipeline", cp.ConePipeline(params))):
    metas = []
    for rep in range(20):
        obj.cloud_handler(msg)
        m = np.zeros(64, np.uint32)
        _abi.check(_abi.lib().cg_debug_large_meta(obj.handle, m.ctypes.data, 64))
        metas.append(m)
    metas = np.array(metas)
    var = [w for w in range(30) if len(set(metas[:, w])) > 1]
    print(name, "K values", sorted(set(metas[:, 19].tolist())), "varying words", var)
    for w in var:
        print("  word", w, sorted(set(metas[:, w].tolist()))[:6])
