"""GPU diagnostic: the C5 frame through the detector, then the PCL voxel sort's leaf list
(cg_debug_large_buffer 3): how many leaves, their sizes, how many exceed the LDS leaf."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cones_perception_amd as cp  # noqa: E402
from cones_perception_amd import _abi  # noqa: E402

params = cp.load_params("simulation")
raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)   # bench C5
det = cp.ConePipeline(params)
d = det.cloud_handler(cp.frame_cloud(raw[0]))
cap, ew, hdr = 2 * 4096 + 64, 5, 8
buf = np.zeros(hdr + 4 * ew * cap, np.uint32)
rc = _abi.lib().cg_debug_large_buffer(det.handle, 3, buf.ctypes.data, buf.nbytes)
nleaf = int(buf[3])
L = buf[hdr + 3 * ew * cap: hdr + 3 * ew * cap + ew * nleaf].reshape(-1, ew)
sz = (L[:, 1] - L[:, 0]).astype(np.int64)
print("rc", rc, "voxels", d.voxels.shape[0], "leaves", nleaf, "sum", int(sz.sum()), "max", int(sz.max()),
      ">2048", int((sz > 2048).sum()), ">1024", int((sz > 1024).sum()), "depth0", int((L[:, 2] == 0).sum()), "depth min", int(L[:, 2].min()) if nleaf else -1)
print("sizes p50/p90/p99", np.percentile(sz, [50, 90, 99]).tolist(), "top", sorted(sz.tolist())[-8:])
