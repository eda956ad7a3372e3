"""GPU, variant library (tools/variants/pqf_stamps.h): lg_pq_flow's per-ticket record on C5's frame
-> per-depth phase times and the critical chain (the ranges whose ends gate the launch's end).
usage: CONES_GPU_LIB=lib_variants/pqfst/libcones_gpu.so python tools/pqf_stamps.py"""
import bisect
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cones_perception_amd as cp  # noqa: E402
from cones_perception_amd import _abi  # noqa: E402
import torch  # noqa: E402

MAXT = 4000
raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
d = torch.from_numpy(raw).cuda()
eng = cp.BatchEngine(cp.load_params("simulation"))
us = lambda x: x / 100.0   # s_memrealtime: 100 MHz


def frame():
    eng.run(d.data_ptr(), 1, raw.shape[1] // 16, 16)
    torch.cuda.synchronize()
    st = np.zeros(128 + 6 * MAXT, np.uint64)
    _abi.check(_abi.lib().cg_debug_large_buffer(eng.handle, 4, st.ctypes.data, st.nbytes))
    r = st[128:].reshape(MAXT, 6).astype(np.uint64)
    t0 = int(r[0, 0])
    live = (r[:, 0] >= t0) & (r[:, 3] & np.uint64((1 << 63) - 1) >= t0) & (r[:, 0] > 0)
    return r, live, t0


per_depth = {}
chains = []
spans = []
for it in range(25):
    r, live, t0 = frame()
    if it < 5:
        continue
    tk = []
    for t in np.nonzero(live)[0]:
        k0, k1, k2, k3, fe, tw = (int(x) for x in r[t])
        f, e, w2, tb = fe & 0xFFFFFFFF, fe >> 32, tw & 0xFFFFFFFF, tw >> 32
        task = (w2 & 0xC0) == 0xC0   # PQF_TASK: partitioned in LDS (its time shows as "swap")
        if (w2 & 64) and not task:
            continue
        pusher = k3 >> 63
        k3 &= (1 << 63) - 1
        swap = bool(w2 & 128) and not task
        if task:
            k1 = k2 = k0
        tk.append(dict(t=int(t), k0=k0 - t0, k1=(k1 - t0) if not swap else None, k2=k2 - t0, k3=k3 - t0, f=f, e=e,
                       depth=(w2 >> 8) & 0xFF, swap=swap, pusher=pusher))
    spans.append(max(x["k3"] for x in tk))
    ranges = {}
    for x in tk:
        g = ranges.setdefault((x["f"], x["e"], x["depth"]), dict(start=1 << 60, split=0, wait=0, end=0, n=0, sw=0))
        g["start"] = min(g["start"], x["k0"])
        if x["k1"] is not None:
            g["split"] = max(g["split"], x["k1"])
        g["wait"] = max(g["wait"], x["k2"])
        g["end"] = max(g["end"], x["k3"])
        g["n"] += 1
        g["sw"] += x["swap"]
    byd = {}
    for (f, e, dp), g in ranges.items():
        byd.setdefault(dp, []).append((f, e, g))

    for lst in byd.values():
        lst.sort(key=lambda z: z[0])
    starts = {dp: [z[0] for z in lst] for dp, lst in byd.items()}

    def parent(f, e, dp):   # (a depth's ranges are disjoint)
        lst = byd.get(dp - 1)
        if not lst:
            return None
        i = bisect.bisect_right(starts[dp - 1], f) - 1
        if i >= 0 and lst[i][0] <= f and e <= lst[i][1]:
            return lst[i]
        return None

    for dp, lst in byd.items():
        pd = per_depth.setdefault(dp, dict(nr=[], pts=[], dur=[], gap=[], split=[], wait=[], swap=[], defer=[]))
        pd["nr"].append(len(lst))
        pd["pts"].append(sum(e - f for f, e, _ in lst))
        for f, e, g in lst:
            pd["dur"].append(g["end"] - g["start"])
            pd["split"].append(g["split"] - g["start"])
            pd["wait"].append(g["wait"] - g["split"])
            pd["swap"].append(g["end"] - g["wait"])
            pd["defer"].append(g["sw"] / max(1, g["n"] - g["sw"]))
            p = parent(f, e, dp)
            if p:
                pd["gap"].append(g["start"] - p[2]["end"])
    # the chain to the last-ending range
    last = max(((f, e, dp, g) for dp, lst in byd.items() for f, e, g in lst), key=lambda z: z[3]["end"])
    ch = []
    f, e, dp, g = last
    while True:
        p = parent(f, e, dp)
        ch.append((dp, e - f, g["n"] - g["sw"], (g["start"] - p[2]["end"]) if p else g["start"], g["split"] - g["start"],
                   g["wait"] - g["split"], g["end"] - g["wait"]))
        if not p:
            break
        f, e, g = p
        dp -= 1
    chains.append(ch[::-1])

med = lambda v: statistics.median(v) if v else float("nan")
print(f"lg_pq_flow span (first ticket taken -> last ticket ends), median {us(med(spans)):.2f} us over {len(spans)} frames")
print("per depth: ranges, points, median range time (first ticket -> last tile's end), its split / wait / swap "
      "phases, parent end -> first ticket taken, deferred swaps per tile, us")
for dp in sorted(per_depth):
    pd = per_depth[dp]
    print(f"  depth {dp:2d}: ranges {med(pd['nr']):6.0f}  points {med(pd['pts']):8.0f}  range {us(med(pd['dur'])):6.2f}  "
          f"split {us(med(pd['split'])):6.2f}  wait {us(med(pd['wait'])):6.2f}  swap {us(med(pd['swap'])):6.2f}  "
          f"gap {us(med(pd['gap'])):6.2f}  deferred {med(pd['defer']):.2f}")
print("critical chain of the median frame (depth, points, tiles, gap from parent end, split, wait, swap), us:")
c = sorted(chains, key=len)[len(chains) // 2]
for dp, npts, nt, gap, sp, wt, sw in c:
    print(f"  depth {dp:2d}  points {npts:8d}  tiles {nt:5d}  gap {us(gap):6.2f}  split {us(sp):6.2f}  wait {us(wt):6.2f}  "
          f"swap {us(sw):6.2f}")
print(f"  chain sum {us(sum(x[3] + x[4] + x[5] + x[6] for x in c)):.2f} us")
