"""ctypes driver for the CPU restatement (oracle/cg_oracle.cpp). Test infrastructure only."""
import ctypes as C
import os

import numpy as np

from cones_perception_amd import Detection, PointCloud2, _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "libcg_oracle.so")
MODE_PIPELINE, MODE_DETECT, MODE_GROUND = 0, 1, 2
ORDER_STABLE, ORDER_PCL = 0, 1
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
        _lib = C.CDLL(ORACLE_SO)
        _lib.oracle_run.restype = C.c_int
        _lib.oracle_run.argtypes = [C.c_void_p] * 2 + [C.c_int, C.c_int] + [C.c_void_p] * 7
        _lib.oracle_atan2f.restype = C.c_float
        _lib.oracle_atan2f.argtypes = [C.c_float, C.c_float]
        _lib.oracle_sector.restype = C.c_int
        _lib.oracle_sector.argtypes = [C.c_float, C.c_float]
    return _lib


def run(params, msg: PointCloud2, mode=MODE_PIPELINE, order=ORDER_STABLE, intensity_offset=None):
    """Run the restatement on one cloud; returns (Detection or ground bytes, header)."""
    n = msg.width * msg.height
    v = msg.view(intensity_offset=intensity_offset)
    cap = max(n, 1)
    hdr = np.zeros(8, np.uint32)
    ground = np.zeros(cap * 8, np.float32) if mode == MODE_GROUND else np.zeros(1, np.float32)
    vox = np.zeros(cap * 4, np.float32)
    lab = np.zeros(cap, np.int32)
    offs = np.zeros(cap + 1, np.int32)
    idx = np.zeros(cap, np.int32)
    cen = np.zeros(cap * 2, np.float32)
    lib().oracle_run(C.addressof(params), C.addressof(v), mode, order, hdr.ctypes.data,
                     ground.ctypes.data, vox.ctypes.data, lab.ctypes.data, offs.ctypes.data,
                     idx.ctypes.data, cen.ctypes.data)
    if mode == MODE_GROUND:
        return ground[: n * 8].view(np.uint8).copy(), hdr
    V, Cn = int(hdr[3]), int(hdr[4])
    nidx = int(offs[Cn]) if Cn else 0
    det = Detection(int(hdr[0]), int(hdr[1]), int(hdr[2]), vox[: V * 4].reshape(V, 4).copy(),
                    lab[:V].copy(), offs[: Cn + 1].copy(), idx[:nidx].copy(),
                    cen[: Cn * 2].reshape(Cn, 2).copy(), int(hdr[5]))
    return det, hdr
