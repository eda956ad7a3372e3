"""How much of the PCL-order voxel sort could be pruned: libstdc++'s
introsort (tests/pb_model.std_sort's control flow) run level by level on a frame's index_vector,
counting per level the partition ranges (> 16 records) and the ones whose order can change a
voxel bit: a range needs libstdc++'s exact permutation only if it holds >= 2 records of one
voxel with >= 3 points (a voxel of <= 2 points sums to the same bits in any order; records of
one voxel in different ranges keep the ranges' order). A level whose ranges are all prunable
could end the sort with a plain key sort. Host model only (CPU)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cones_perception_amd as cp  # noqa: E402
import np_reference as R  # noqa: E402
from pb_model import THRESH, key, move_median_to_first, _lg  # noqa: E402

F32 = np.float32


def index_vector(pts, prm):
    """(idx << 32 | i) records of the detector's finite survivors, in cloud order."""
    inv = np.array([F32(1.0) / F32(prm[f"voxel_filter_leaf_size_{a}"]) for a in "xyz"], F32)
    fin = np.isfinite(pts[:, :3]).all(axis=1)
    P = pts[fin]
    if not len(P):
        return []
    mn = P[:, :3].min(axis=0)
    mx = P[:, :3].max(axis=0)
    min_b = np.floor(mn * inv).astype(np.int64)
    max_b = np.floor(mx * inv).astype(np.int64)
    div = max_b - min_b + 1
    ijk = (np.floor(P[:, :3] * inv) - min_b.astype(F32)).astype(np.int64)
    idx = (ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * (div[0] * div[1])) & 0xFFFFFFFF
    return [(int(k) << 32) | i for i, k in enumerate(idx)]


def levels(recs):
    """Per introsort level: (ranges > THRESH, of them needing the exact permutation)."""
    f = list(recs)
    n = len(f)
    cnt = {}
    for r in f:
        cnt[key(r)] = cnt.get(key(r), 0) + 1
    hot = {k for k, c in cnt.items() if c >= 3}
    out = []
    cur = [(0, n, 2 * _lg(n))] if n > THRESH else []
    while cur:
        nxt, tot, need = [], 0, 0
        for first, last, depth in cur:
            tot += 1
            seen = {}
            sens = False
            for r in f[first:last]:
                k = key(r)
                if k in hot:
                    seen[k] = seen.get(k, 0) + 1
                    if seen[k] >= 2:
                        sens = True
                        break
            need += sens
            if depth == 0:
                continue
            move_median_to_first(f, first, first + 1, first + (last - first) // 2, last - 1)
            lo, hi, p = first + 1, last, key(f[first])
            while True:
                while key(f[lo]) < p:
                    lo += 1
                hi -= 1
                while p < key(f[hi]):
                    hi -= 1
                if not lo < hi:
                    break
                f[lo], f[hi] = f[hi], f[lo]
                lo += 1
            for a, b in ((first, lo), (lo, last)):
                if b - a > THRESH:
                    nxt.append((a, b, depth - 1))
        out.append((tot, need))
        cur = nxt
    return out


def main():
    prm = {k: getattr(cp.load_params("simulation"), k) for k in
           ("level_threshold", "distance_treshold_max", "distance_treshold_min", "angle_threshold",
            "voxel_filter_leaf_size_x", "voxel_filter_leaf_size_y", "voxel_filter_leaf_size_z", "default_lowest_point")}
    which = sys.argv[1] if len(sys.argv) > 1 else "c3"
    if which == "c3":
        raw = cp.synth_frames(64, first_frame=0, rings=64, cols=1024)
    else:
        raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
    agg = {}
    for fr in raw:
        pts = fr.view(F32).reshape(-1, 4)
        g, _ = R.ground_remove(pts, prm["default_lowest_point"])
        s = R.filter_points_position(g, prm)
        for lv, (t, nd) in enumerate(levels(index_vector(s, prm))):
            a = agg.setdefault(lv, [0, 0, 0])
            a[0] += t; a[1] += nd; a[2] += nd == 0
    print(f"{which}: {len(raw)} frames")
    print("level  ranges  need-exact  prunable  frames-with-level-all-prunable")
    for lv in sorted(agg):
        t, nd, allp = agg[lv]
        print(f"{lv:5d} {t:7d} {nd:11d} {t - nd:9d} {allp:6d}")


if __name__ == "__main__":
    main()
