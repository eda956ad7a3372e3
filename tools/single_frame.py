"""Diagnostic: C2 single-frame latency of the synchronous drop-in call (ConePipeline.cloud_handler:
PointCloud2 bytes in host memory -> results on the host), by route (0: frame kernel, 1: the
large-frame path's multi-workgroup front, 3: the frame kernel in one workgroup, 4: pass 1 in one
workgroup per 4,096-point chunk with the input copied by DMA; 0: the same with the chunks
read by the kernel from pinned memory), with a host memcpy of the frame for scale."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cones_perception_amd as cp  # noqa: E402
from cones_perception_amd import _abi  # noqa: E402

params = cp.load_params("simulation")
raw = cp.synth_frames(8, first_frame=0, rings=64, cols=1024)
msgs = [cp.frame_cloud(raw[i]) for i in range(8)]
dst = np.empty_like(raw[0])
t0 = time.perf_counter()
for i in range(200):
    np.copyto(dst, raw[i % 8])
print(f"host memcpy of one 1 MiB frame: {(time.perf_counter() - t0) / 200 * 1e6:.1f} us")
for route in (0, 4, 3, 1):
    pipe = cp.ConePipeline(params, device=0)
    _abi.check(_abi.lib().cg_debug_route(pipe.handle, route))
    for i in range(20):
        pipe.cloud_handler(msgs[i % 8])
    t0 = time.perf_counter()
    for i in range(200):
        pipe.cloud_handler(msgs[i % 8])
    print(f"route {route}: {(time.perf_counter() - t0) / 200 * 1e6:.1f} us per synchronous frame call")

# the bare C-ABI call (no Python result objects): what a C++ node pays
import ctypes as C  # noqa: E402
pipe = cp.ConePipeline(params, device=0)
views = [m.view() for m in msgs]
r = _abi.cg_detect_result()
lib = _abi.lib()
for i in range(20):
    _abi.check(lib.cg_pipeline(pipe.handle, C.byref(views[i % 8]), C.byref(r)))
t0 = time.perf_counter()
for i in range(200):
    lib.cg_pipeline(pipe.handle, C.byref(views[i % 8]), C.byref(r))
print(f"bare cg_pipeline call: {(time.perf_counter() - t0) / 200 * 1e6:.1f} us")
