"""CPU: how many of C5's partition levels carry work. The C5 frame's index_vector keys (numpy restatement,
tests/np_reference.py), then libstdc++'s introsort level by level: per level, the ranges longer than the cut
(LG_PCL_CUT, default 2,048) that the next level partitions.  usage: python tools/c5_levels.py [cut]"""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import cones_perception_amd as cp
import np_reference as R
prm = cp.load_params("simulation")
prm = {k: getattr(prm, k) for k in dir(prm) if not k.startswith("_")} if not isinstance(prm, dict) else prm
raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
msg = cp.frame_cloud(raw[0])
pts = np.frombuffer(bytes(msg.data), np.float32).reshape(-1, 4) if hasattr(msg, "data") else None
g, K = R.ground_remove(pts, prm["default_lowest_point"])
f = R.filter_points_position(g, prm)
inv = np.array([np.float32(1.0) / np.float32(prm[f"voxel_filter_leaf_size_{a}"]) for a in "xyz"], np.float32)
fin = np.isfinite(f[:, :3]).all(axis=1); P = f[fin]
mn = P[:, :3].min(axis=0); mx = P[:, :3].max(axis=0)
min_b = np.floor(mn * inv).astype(np.int64); max_b = np.floor(mx * inv).astype(np.int64); div = max_b - min_b + 1
ijk = (np.floor(P[:, :3] * inv) - min_b.astype(np.float32)).astype(np.int64)
idx = ((ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * (div[0] * div[1])) & 0xFFFFFFFF).tolist()
print("M", len(idx), "V", len(set(idx)))
# libstdc++ introsort, level-synchronous: record ranges partitioned per level
f_ = list(idx); n = len(f_)
def lg(n): return n.bit_length() - 1
cur = [(0, n, 2 * lg(n))]
lvl = 0
CUT = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
while cur:
    big = [r for r in cur if r[1] - r[0] > CUT]
    print(f"level {lvl}: ranges {len(cur)} cut>{CUT}: {len(big)} records {sum(e-s for s,e,_ in big)} max {max(e-s for s,e,_ in cur)}")
    nxt = []
    for (first, last, depth) in big:
        a, b, c = first + 1, first + (last - first) // 2, last - 1
        ka, kb, kc = f_[a], f_[b], f_[c]
        if ka < kb:
            m = b if kb < kc else (c if ka < kc else a)
        elif ka < kc: m = a
        else: m = c if kb < kc else b
        f_[first], f_[m] = f_[m], f_[first]
        lo, hi, p = first + 1, last, f_[first]
        while True:
            while f_[lo] < p: lo += 1
            hi -= 1
            while p < f_[hi]: hi -= 1
            if not lo < hi: break
            f_[lo], f_[hi] = f_[hi], f_[lo]; lo += 1
        nxt += [(first, lo, depth - 1), (lo, last, depth - 1)]
    cur = nxt; lvl += 1
    if lvl > 30: break
