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
        _lib.oracle_run_search.restype = C.c_int
        _lib.oracle_run_search.argtypes = [C.c_void_p] * 2 + [C.c_int, C.c_int, C.c_int] + [C.c_void_p] * 7
        _lib.oracle_flann_check.restype = C.c_int
        _lib.oracle_flann_check.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        _lib.oracle_flann_radius_all.restype = C.c_uint32
        _lib.oracle_flann_radius_all.argtypes = [C.c_void_p, C.c_uint32, C.c_float, C.c_void_p, C.c_void_p,
                                                 C.c_uint32]
        _lib.oracle_atan2f.restype = C.c_float
        _lib.oracle_atan2f.argtypes = [C.c_float, C.c_float]
        _lib.oracle_sector.restype = C.c_int
        _lib.oracle_sector.argtypes = [C.c_float, C.c_float]
        _lib.oracle_recrop.restype = C.c_uint32
        _lib.oracle_recrop.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_uint32, C.c_void_p,
                                       C.c_void_p, C.c_uint32]
        _lib.oracle_node_create.restype = C.c_void_p
        _lib.oracle_node_create.argtypes = [C.c_int, C.c_int, C.c_double]
        _lib.oracle_node_destroy.restype = None
        _lib.oracle_node_destroy.argtypes = [C.c_void_p]
        _lib.oracle_node_step.restype = C.c_int
        _lib.oracle_node_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_uint32,
                                          SERVICE_FN, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
    return _lib


SERVICE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_uint32), C.c_uint32,
                         C.POINTER(C.c_int32), C.c_uint32)


def recrop(params, msg: PointCloud2, mode, centres, intensity_offset=None):
    """get_reconstructed_cone over the whole cloud of msg (mode: MODE_PIPELINE = the groundless
    cloud, MODE_DETECT = the detector input): one (n, 4) array per centre."""
    v = msg.view(intensity_offset=intensity_offset)
    cen = np.ascontiguousarray(np.asarray(centres, np.float32).reshape(-1, 2))
    n = cen.shape[0]
    offs = np.zeros(n + 1, np.uint32)
    cap = 1 << 16
    while True:
        pts = np.zeros((cap, 4), np.float32)
        tot = lib().oracle_recrop(C.addressof(params), C.addressof(v), mode, cen.ctypes.data, n,
                                  offs.ctypes.data, pts.ctypes.data, cap)
        if tot <= cap:
            break
        cap = int(tot)
    return [pts[offs[i]:offs[i + 1]].copy() for i in range(n)]


class Node:
    """The restated node state after the hot path (tracking + colour clouds)."""

    def __init__(self, classify_colors=True, use_points_buffer=False, matching=0.5):
        self._n = lib().oracle_node_create(int(classify_colors), int(use_points_buffer), matching)

    def __del__(self):
        if getattr(self, "_n", None):
            lib().oracle_node_destroy(self._n)
            self._n = None

    def step(self, params, msg: PointCloud2, mode, centroids, service, intensity_offset=None):
        """service(list of (n_k, 4) xyzi crops, request order) -> the response's colours (a list,
        possibly shorter than the request), or None for a failed call. Returns the four colour
        clouds as (k, 2) arrays."""
        v = msg.view(intensity_offset=intensity_offset)
        cen = np.ascontiguousarray(np.asarray(centroids, np.float32).reshape(-1, 2))

        def cb(_ctx, ptr, offs, n, out, cap):
            tot = offs[n] if n else 0
            pts = np.ctypeslib.as_array(ptr, (tot * 4,)).reshape(tot, 4).copy() if tot else np.zeros((0, 4), np.float32)
            crops = [pts[offs[k]:offs[k + 1]] for k in range(n)]
            resp = service(crops)
            if resp is None:
                return -1
            resp = [int(c) for c in resp]
            if len(resp) > cap:
                return cap
            for k, c in enumerate(resp):
                out[k] = c
            return len(resp)

        fn = SERVICE_FN(cb)
        cap = max(cen.shape[0], 1)
        counts = np.zeros(4, np.uint32)
        xy = np.zeros((4, cap, 2), np.float32)
        rc = lib().oracle_node_step(self._n, C.addressof(params), C.addressof(v), mode,
                                    cen.ctypes.data if cen.size else None, cen.shape[0], fn, None,
                                    counts.ctypes.data, xy.ctypes.data, cap)
        if rc != 0:
            raise ValueError("colour service response longer than the request, or a colour out of range")
        return [xy[i, : counts[i]].copy() for i in range(4)]


def server(crops, classify):
    """The reference's service handler (scripts/color_classifier_server.py:81-124) around a
    per-crop classifier: empty crops get no answer (`continue`, lines 83-84), so the response
    lists the non-empty crops' colours in request order."""
    return [int(classify(c)) for c in crops if len(c)]


SEARCH_EXACT, SEARCH_FLANN = 0, 1
FLANN_STATS = ("voxels", "queries_differ", "pairs_missed", "pairs_extra", "near_tolerance_pairs",
               "near_tolerance_inside", "clusters_equal", "clusters_exact", "clusters_flann", "closest_inside_ulps")


def flann_check(params, msg: PointCloud2, mode=MODE_PIPELINE, order=ORDER_PCL, intensity_offset=None) -> dict:
    """oracle_flann_check on one cloud: FLANN 1.9.1's own tree and search (restated) against the
    exact radius predicate, for every voxel as a query, and both clusterings."""
    v = msg.view(intensity_offset=intensity_offset)
    st = np.zeros(10, np.uint32)
    lib().oracle_flann_check(C.addressof(params), C.addressof(v), mode, order, st.ctypes.data)
    return dict(zip(FLANN_STATS, (int(x) for x in st)))


def flann_radius_all(xyz, r2):
    """FLANN's radius search (restated) with every point of xyz (n, 3) as the query: a list of
    neighbour index arrays, each sorted by (distance, index)."""
    xyz = np.ascontiguousarray(np.asarray(xyz, np.float32).reshape(-1, 3))
    n = xyz.shape[0]
    counts = np.zeros(max(n, 1), np.uint32)
    cap = max(64 * n, 1)
    while True:
        idx = np.zeros(cap, np.int32)
        tot = lib().oracle_flann_radius_all(xyz.ctypes.data, n, float(r2), counts.ctypes.data, idx.ctypes.data, cap)
        if tot <= cap:
            break
        cap = int(tot)
    offs = np.concatenate([[0], np.cumsum(counts[:n])]).astype(np.int64)
    return [idx[offs[i]:offs[i + 1]].copy() for i in range(n)]


def run(params, msg: PointCloud2, mode=MODE_PIPELINE, order=ORDER_PCL, intensity_offset=None, search=SEARCH_EXACT):
    """Run the restatement on one cloud; returns (Detection or ground bytes, header). order:
    ORDER_PCL (default) sums each voxel in PCL's std::sort order, as the reference and the device
    do; ORDER_STABLE in ascending point order (the numpy restatement's and the halo form's).
    search: SEARCH_EXACT (default) clusters with the exact L2_Simple radius predicate,
    SEARCH_FLANN with FLANN 1.9.1's own tree and pruning (restated)."""
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
    lib().oracle_run_search(C.addressof(params), C.addressof(v), mode, order, search, hdr.ctypes.data,
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
