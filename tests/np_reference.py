"""Independent numpy/scipy restatement of the reference hot path (test infrastructure only).

Written separately from oracle/cg_oracle.cpp, with different machinery (vectorised numpy
float32/float64, scipy connected components instead of a kd-tree BFS, numpy lexsort instead of
std::sort), so that the two restatements agreeing bit for bit stands in for the PCL/ROS build
that cannot exist here. Each step cites the reference line it follows.
libm's atan2f is called through ctypes: numpy's own arctan2 is not glibc's.
"""
import ctypes

import numpy as np
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components

_libm = ctypes.CDLL("libm.so.6")
_libm.atan2f.restype = ctypes.c_float
_libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
F32 = np.float32


def atan2f(y, x):
    return np.array([_libm.atan2f(float(a), float(b)) for a, b in zip(y, x)], dtype=F32)


def sector_index(a):
    """src/ground_removal.cpp:61-64 with the 17th bin (G3) and a NaN bin (17)."""
    sec = F32((360 // 16) * np.pi / 180)
    wrapped = np.where(a < 0, (a.astype(np.float64) + 2 * np.pi).astype(F32), a)
    with np.errstate(invalid="ignore"):
        q = np.floor(wrapped / sec)
    s = np.where(np.isnan(q), 17, q).astype(np.int64)
    return s


def ground_remove(pts, default_low):
    """src/ground_removal.cpp:56-79 -> (N x 4 groundless cloud, K)."""
    n = pts.shape[0]
    if n == 0:
        return pts.copy(), 0
    x, y, z = pts[:, 0], pts[:, 1], pts[:, 2]
    s = sector_index(atan2f(y, x))
    low = np.full(18, F32(default_low), F32)
    for b in range(17):
        zb = z[(s == b) & ~np.isnan(z)]
        if zb.size:
            low[b] = min(low[b], zb.min())
    thr = low[s].astype(np.float64) + 0.1
    with np.errstate(invalid="ignore"):
        keep = ~(z.astype(np.float64) < thr)
    kept = pts[keep]
    out = np.zeros_like(pts)
    out[: kept.shape[0]] = kept
    return out, int(kept.shape[0])


def filter_points_position(pts, prm):
    """src/cone_detection.cpp:189-204 (euclidan_dist: utils.cpp:32-34)."""
    if pts.shape[0] == 0:
        return pts
    x64, y64, z64 = (pts[:, i].astype(np.float64) for i in range(3))
    d = np.sqrt((x64 * x64 + y64 * y64) + z64 * z64).astype(F32).astype(np.float64)
    a = atan2f(pts[:, 1], pts[:, 0]).astype(np.float64)
    th = prm["angle_threshold"] * np.pi / 180
    nth = -prm["angle_threshold"] * np.pi / 180
    with np.errstate(invalid="ignore"):
        rm = (z64 < prm["level_threshold"]) | (d > prm["distance_treshold_max"]) | \
             (d < prm["distance_treshold_min"]) | (nth >= a) | (a >= th)
    return pts[~rm]


def voxel_grid(pts, prm):
    """pcl::VoxelGrid<PointXYZI> (PCL 1.10) with per-voxel sums in ascending point order."""
    inv = np.array([F32(1.0) / F32(prm[f"voxel_filter_leaf_size_{a}"]) for a in "xyz"], F32)
    fin = np.isfinite(pts[:, :3]).all(axis=1)
    if not fin.any():
        return np.zeros((0, 4), F32), False
    P = pts[fin]
    pos = np.nonzero(fin)[0]
    mn, mx = P[:, :3].min(axis=0), P[:, :3].max(axis=0)
    span = ((mx - mn) * inv).astype(F32)
    dims = np.floor(span.astype(np.float64)).astype(np.int64) + 1
    if float(dims[0]) * float(dims[1]) * float(dims[2]) > 2147483647.0:
        return pts.copy(), True
    min_b = np.floor(mn * inv).astype(np.int64)
    max_b = np.floor(mx * inv).astype(np.int64)
    div = max_b - min_b + 1
    ijk = (np.floor(P[:, :3] * inv) - min_b.astype(F32)).astype(np.int64)
    idx = (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * (div[0] * div[1])) & 0xFFFFFFFF
    order = np.lexsort((pos, idx))
    idx_s = idx[order]
    heads = np.r_[True, idx_s[1:] != idx_s[:-1]]
    starts = np.nonzero(heads)[0]
    ends = np.r_[starts[1:], idx_s.size]
    out = np.zeros((starts.size, 4), F32)
    for v, (s0, e0) in enumerate(zip(starts, ends)):
        acc = np.zeros(4, F32)
        for j in order[s0:e0]:
            acc = (acc + P[j]).astype(F32)
        out[v] = acc / F32(e0 - s0)
    return out, False


def euclidean_clusters(vox, min_size, max_size):
    """Connected components of d2 = fl(fl(dx^2 + dy^2) + dz^2) < r2 (FLANN L2_Simple), PCL's
    size filter (unsigned compare) and (size desc, seed asc) order."""
    cone_h, cone_w = F32(0.325), F32(0.228)
    tol = F32(np.sqrt(np.float64(cone_h) ** 2 + np.float64(cone_w) ** 2))
    r2 = F32(np.float64(tol) * np.float64(tol))
    V = vox.shape[0]
    if V == 0:
        return []
    p = vox[:, :3].astype(F32)
    d = p[:, None, :] - p[None, :, :]
    d2 = ((d[..., 0] * d[..., 0]) + (d[..., 1] * d[..., 1])) + (d[..., 2] * d[..., 2])
    with np.errstate(invalid="ignore"):
        adj = d2 < r2
    np.fill_diagonal(adj, False)
    ii, jj = np.nonzero(adj)
    g = coo_matrix((np.ones(ii.size, np.int8), (ii, jj)), shape=(V, V))
    _, lab = connected_components(g, directed=False)
    comps = {}
    for v in range(V):
        comps.setdefault(lab[v], []).append(v)
    lo, hi = min_size & 0xFFFFFFFF, max_size & 0xFFFFFFFF
    kept = [sorted(c) for c in comps.values() if lo <= len(c) <= hi]
    kept.sort(key=lambda c: (-len(c), c[0]))
    return kept


def centroids(vox, clusters, ext):
    """src/cone_detection.cpp:261-279 (x sum starts at 0)."""
    out = np.zeros((len(clusters), 2), F32)
    for k, c in enumerate(clusters):
        x = F32(0.0)
        y = F32(0.0)
        for i in c:
            x = F32(x + vox[i, 0])
            y = F32(y + vox[i, 1])
        px, py = F32(x / F32(len(c))), F32(y / F32(len(c)))
        ln = F32(np.sqrt((np.float64(px) ** 2 + np.float64(py) ** 2) + 0.0))
        with np.errstate(invalid="ignore", divide="ignore"):
            out[k, 0] = F32(np.float64(px) + np.float64(F32(px / ln)) * ext)
            out[k, 1] = F32(np.float64(py) + np.float64(F32(py / ln)) * ext)
    return out


def pipeline(pts, prm, ground=True):
    """ground_removal (optional) -> filter -> voxel -> clusters -> centroids."""
    K = pts.shape[0]
    if ground:
        pts, K = ground_remove(pts, prm["default_lowest_point"])
    f = filter_points_position(pts, prm)
    vox, passthrough = voxel_grid(f, prm)
    cl = euclidean_clusters(vox, prm["min_cluster_size"], prm["max_cluster_size"])
    return {"K": K, "M": f.shape[0], "vox": vox, "passthrough": passthrough, "clusters": cl,
            "centroids": centroids(vox, cl, prm["cone_position_extension_length"])}
