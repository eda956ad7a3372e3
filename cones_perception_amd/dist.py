"""Frame-batch sharding across GPUs (one process per GPU, torch.distributed; "nccl" = RCCL).

Frames are independent units, so the steady-state path has no data-path
collective: rank r owns frames [r*F, (r+1)*F) already resident in its HBM, and only the
timing (max over ranks) and the small per-frame result headers cross ranks. For the C4
composition the north star describes (a root holding the whole batch), `scatter_frames`
moves each rank's share with one scatter and `gather_headers` brings the per-frame results
back with one gather; over xGMI that is one point-to-point transfer per peer.
"""
import os

import torch
import torch.distributed as dist


# Collectives run even at world size 1 when forced (CG_FORCE_COLLECTIVES=1 or
# force_collectives()): one rank under RCCL then exercises every device-tensor collective of
# the multi-GPU paths on a one-GPU box (tests/test_gpu_rccl.py, bench.py --scatter).
_FORCE = os.environ.get("CG_FORCE_COLLECTIVES", "0") == "1"


def force_collectives(on: bool = True) -> None:
    global _FORCE
    _FORCE = bool(on)


def world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def frame_range(rank: int, frames_per_rank: int) -> range:
    """Global frame indices owned by `rank` (weak scaling: fixed frames per rank)."""
    return range(rank * frames_per_rank, (rank + 1) * frames_per_rank)


def max_over_ranks(value: float, device) -> float:
    if not _distributed():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def scatter_frames(all_frames, frames_per_rank: int, frame_bytes: int, device, src: int = 0):
    """Root holds (world * F, frame_bytes) uint8 frames; every rank receives its (F, frame_bytes)."""
    ws = dist.get_world_size()
    out = torch.empty((frames_per_rank, frame_bytes), dtype=torch.uint8, device=device)
    chunks = list(all_frames.chunk(ws, dim=0)) if dist.get_rank() == src else None
    dist.scatter(out, chunks, src=src)
    return out


def gather_headers(headers, dst: int = 0):
    """Gather each rank's (F, 8) int32 per-frame result headers to `dst` as (world * F, 8)."""
    ws = dist.get_world_size()
    bufs = [torch.empty_like(headers) for _ in range(ws)] if dist.get_rank() == dst else None
    dist.gather(headers, bufs, dst=dst)
    return torch.cat(bufs, 0) if bufs is not None else None


# ---------------------------------------------------------------------------------------------
# C5: one large frame tiled across ranks (include/cones_gpu.h, cg_tile_*). Tiles are contiguous
# point-index ranges; for a column-major spinning LiDAR (point = column * rings + ring) a range
# is an azimuth wedge, i.e. a spatial tile. The exchange steps are two small all-reduces (the
# 18 sector-minimum keys with the used-bin mask, then counts and VoxelGrid bounds) and one
# gather of the survivors (a few percent of the points) to the rank that runs the backend.

def tile_range(n_total: int, rank: int, world_size: int):
    """Points [lo, hi) of rank's tile."""
    per = (n_total + world_size - 1) // world_size
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


def _distributed() -> bool:
    return dist.is_initialized() and (dist.get_world_size() > 1 or _FORCE)


def _coll_device(device):
    """Collectives run on the GPU under RCCL ("nccl") and on the host under gloo."""
    return device if dist.get_backend() == "nccl" else torch.device("cpu")


def merge_tile_keys(keys, device):
    """keys: uint32[19] of this rank -> merged uint32[19]: words 0-17 MIN (order-preserving
    sector-minimum keys), word 18 bitwise OR of the used-bin masks. One MIN all-reduce: RCCL
    has no bitwise reduction, and OR over ranks of a bit is -MIN(-bit)."""
    import numpy as np
    if not _distributed():
        return np.asarray(keys, np.uint32).copy()
    cd = _coll_device(device)
    v = np.empty(18 + 32, np.int64)
    v[:18] = np.asarray(keys[:18], np.int64)
    v[18:] = -((int(keys[18]) >> np.arange(32)) & 1)
    t = torch.from_numpy(v).to(cd)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    r = t.cpu().numpy()
    out = np.zeros(19, np.uint32)
    out[:18] = r[:18].astype(np.uint32)
    out[18] = int(sum(1 << b for b in range(32) if r[18 + b] < 0))
    return out


def merge_tile_counts(counts, device, per_rank: bool = False):
    """counts: uint32[9] (K, survivors, finite survivors, bounds-min keys x3, bounds-max keys x3)
    -> merged: SUM, SUM, SUM, MIN x3, MAX x3. One all-gather, reduced on the host; with
    per_rank, also every rank's survivor count (the sizes gather_survivors needs)."""
    import numpy as np
    if not _distributed():
        out = np.asarray(counts, np.uint32).copy()
        return (out, [int(out[1])]) if per_rank else out
    cd = _coll_device(device)
    ws = dist.get_world_size()
    t = torch.from_numpy(np.asarray(counts, np.int64).copy()).to(cd)
    parts = [torch.empty_like(t) for _ in range(ws)]
    dist.all_gather(parts, t)
    c = torch.stack(parts).cpu().numpy()
    out = np.concatenate([c[:, :3].sum(0), c[:, 3:6].min(0), c[:, 6:9].max(0)]).astype(np.uint32)
    return (out, [int(x) for x in c[:, 1]]) if per_rank else out


def _u32_bits(x):
    """int64 values in [0, 2^32) -> the same bits as int32 (the C-ABI's uint32 words)."""
    return (x - ((x >= 2 ** 31).to(torch.int64) << 32)).to(torch.int32)


def merge_tile_keys_dev(keys, device):
    """merge_tile_keys on the device: keys int32[19] (uint32 bits) of this rank, on `device`, ->
    merged int32[19] on `device`. One MIN all-reduce (on the GPU under RCCL, through the host
    under gloo); one rank: the keys themselves."""
    if not _distributed():
        return keys
    cd = _coll_device(device)
    k = keys.to(torch.int64) & 0xFFFFFFFF
    sh = torch.arange(32, device=keys.device, dtype=torch.int64)
    v = torch.cat([k[:18], -((k[18] >> sh) & 1)]).to(cd)
    dist.all_reduce(v, op=dist.ReduceOp.MIN)
    v = v.to(keys.device)
    word18 = ((v[18:] < 0).to(torch.int64) << sh).sum().view(1)
    return _u32_bits(torch.cat([v[:18], word18]))


def merge_tile_counts_dev(counts, device):
    """merge_tile_counts for counts int32[9] (uint32 bits) on `device`: one all-gather, then
    one read to the host (the survivor counts size the survivor gather). Returns (merged
    uint32[9] numpy, every rank's survivor count)."""
    import numpy as np
    cd = _coll_device(device)
    t = (counts.to(torch.int64) & 0xFFFFFFFF).to(cd)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    c = torch.stack(parts).cpu().numpy()
    out = np.concatenate([c[:, :3].sum(0), c[:, 3:6].min(0), c[:, 6:9].max(0)]).astype(np.uint32)
    return out, [int(x) for x in c[:, 1]]


def gather_survivors(points, index, device, dst: int = 0, sizes=None):
    """Gather every rank's survivors ((n, 4) float32 and (n,) int32, any n) to dst as one
    concatenation in rank order (the backend does not depend on the order). Others get None.
    The index rides as a fifth float32 column (bit-cast), so it is one all-gather when `sizes`
    (every rank's n, from merge_tile_counts(per_rank=True)) is known, two otherwise."""
    if not _distributed():
        return points.to(device).contiguous(), index.to(device).contiguous()
    cd = _coll_device(device)
    ws = dist.get_world_size()
    if sizes is None:
        n = torch.tensor([points.shape[0]], dtype=torch.int64, device=cd)
        parts = [torch.zeros_like(n) for _ in range(ws)]
        dist.all_gather(parts, n)
        sizes = [int(x.item()) for x in parts]
    m = max(1, max(sizes))
    rows = torch.zeros((m, 5), dtype=torch.float32, device=cd)
    k = points.shape[0]
    rows[:k, :4] = points.to(cd)
    rows[:k, 4] = index.to(cd).view(torch.float32)
    parts = [torch.empty_like(rows) for _ in range(ws)]
    dist.all_gather(parts, rows)
    if dist.get_rank() != dst:
        return None, None
    allr = torch.cat([parts[r][: sizes[r]] for r in range(ws)], 0).to(device)
    return allr[:, :4].contiguous(), allr[:, 4].contiguous().view(torch.int32)


def _tile_front_decide(engine, d_tile_ptr, first, n, n_total, device, point_step, offsets):
    """Steps 1-2 of the tile protocol plus the rank's survivors: (merged counts, every rank's
    survivor count, survivor points (ns, 4), frame indices (ns,))."""
    import ctypes as C
    import numpy as np
    from . import _abi
    lib, h = _abi.lib(), engine.handle
    t = _abi.cg_tile(d_tile_ptr, first, n, n_total, point_step, *offsets)
    keys = np.zeros(_abi.CG_TILE_KEYS, np.uint32)
    _abi.check(lib.cg_tile_front(h, C.byref(t), keys.ctypes.data))
    merged = merge_tile_keys(keys, device)
    counts = np.zeros(_abi.CG_TILE_COUNTS, np.uint32)
    _abi.check(lib.cg_tile_decide(h, merged.ctypes.data, counts.ctypes.data))
    ns = int(counts[1])
    sp = torch.empty((max(ns, 1), 4), dtype=torch.float32, device=device)
    si = torch.empty((max(ns, 1),), dtype=torch.int32, device=device)
    _abi.check(lib.cg_tile_survivors(h, sp.data_ptr(), si.data_ptr(), sp.shape[0]))
    total, sizes = merge_tile_counts(counts, device, per_rank=True)
    return total, sizes, sp[:ns], si[:ns]


def _tile_front_decide_dev(engine, d_tile_ptr, first, n, n_total, device, point_step, offsets):
    """_tile_front_decide with the keys and counts on the device (cg_tile_*_async on the
    engine's tile stream, as the gather form): one host read, of the merged counts (every
    rank's survivor count sizes its survivor buffer), and the survivors complete on return
    (the cg_halo_* calls run on the handle's own stream)."""
    import ctypes as C
    import numpy as np
    from . import _abi
    lib, h = _abi.lib(), engine.handle
    st = _tile_stream(engine, device)
    st.wait_stream(torch.cuda.current_stream(device))   # the tile's points
    s = st.cuda_stream
    with torch.cuda.stream(st):
        t = _abi.cg_tile(d_tile_ptr, first, n, n_total, point_step, *offsets)
        keys = torch.empty(_abi.CG_TILE_KEYS, dtype=torch.int32, device=device)
        _abi.check(lib.cg_tile_front_async(h, C.byref(t), keys.data_ptr(), s))
        merged = merge_tile_keys_dev(keys, device)
        counts = torch.empty(_abi.CG_TILE_COUNTS, dtype=torch.int32, device=device)
        _abi.check(lib.cg_tile_decide_async(h, merged.data_ptr(), counts.data_ptr(), s))
        if _distributed():
            total, sizes = merge_tile_counts_dev(counts, device)
            ns = sizes[dist.get_rank()]
        else:
            total = counts.cpu().numpy().view(np.uint32).copy()
            sizes = [int(total[1])]
            ns = sizes[0]
        sp = torch.empty((max(ns, 1), 4), dtype=torch.float32, device=device)
        si = torch.empty((max(ns, 1),), dtype=torch.int32, device=device)
        _abi.check(lib.cg_tile_survivors_async(h, sp.data_ptr(), si.data_ptr(), ns, s))
    st.synchronize()
    return total, sizes, sp[:ns], si[:ns]


def run_tiled_frame(engine, d_tile_ptr: int, first: int, n: int, n_total: int, device, point_step: int = 16,
                    offsets=(0, 4, 8, 12), dst: int = 0, halo: bool = False, fetch: bool = True):
    """Pipeline one frame of n_total points whose points [first, first + n) are at d_tile_ptr
    on this rank's GPU. `engine` is a cones_perception_amd.BatchEngine (the handle). Returns the
    frame's Detection on dst (bit-identical to the single-GPU call on the whole frame).
    halo=False gathers the survivors to dst, which runs the backend; halo=True tiles the
    backend too (run_halo_backend: voxel slabs, a halo exchange between neighbouring slabs).
    fetch=False leaves the result in the handle's device buffers (engine.fetch(0) reads it)
    and returns True on dst."""
    from . import _abi
    if halo and not _distributed():
        # one rank: one slab and no halo, so the slab's backend is the frame's, with its voxel
        # sums in point order as every slab's; it runs on the survivors where decide left them
        # (the gather form's one-rank path), with no survivor copy, plan or records
        last_halo_stats.clear()
        last_halo_stats.update(slabs=1, slab_w=None, band=None, survivors=None, voxels=None, halo_sent=0,
                               halo_received=0, pairs=0,
                               path="one rank, no collectives: the gather form's backend in point order "
                                    "(no cg_halo_* call)")
        return _run_tiled_gather(engine, d_tile_ptr, first, n, n_total, device, point_step, offsets, dst, fetch,
                                 order=_abi.CG_VOXEL_ORDER_POINT)
    if halo:
        total, sizes, sp, si = _tile_front_decide_dev(engine, d_tile_ptr, first, n, n_total, device, point_step,
                                                      offsets)
        det = run_halo_backend(engine, total, sp, si, n_total, device, dst, fetch=fetch, sizes=sizes)
        if det is not False:
            return det
        gp, gi = gather_survivors(sp, si, device, dst, sizes=sizes)
        if _distributed() and dist.get_rank() != dst:
            return None
        _abi.check(_abi.lib().cg_tile_backend(engine.handle, gp.data_ptr(), gi.data_ptr(), int(gp.shape[0]),
                                              total.ctypes.data, n_total))
        return engine.fetch(0) if fetch else True
    return _run_tiled_gather(engine, d_tile_ptr, first, n, n_total, device, point_step, offsets, dst, fetch)


def _tile_stream(engine, device):
    """One torch stream per engine for the gather form: the C-ABI calls, the torch ops and the
    collectives of a frame all run on it, in order, with no host synchronisation."""
    st = getattr(engine, "_tile_stream", None)
    if st is None:
        st = torch.cuda.Stream(device)
        engine._tile_stream = st
    return st


def _run_tiled_gather(engine, d_tile_ptr, first, n, n_total, device, point_step, offsets, dst, fetch, order=None):
    """The gather form with the keys and counts on the device (cg_tile_*_async): the keys
    merge with a MIN all-reduce on the GPU; one rank (its tile the whole frame) runs the
    backend on its own survivors where they are; several ranks merge the counts with one
    all-gather, read back once for the survivor counts, and gather the survivors to dst."""
    import ctypes as C
    from . import _abi
    lib, h = _abi.lib(), engine.handle
    st = _tile_stream(engine, device)
    caller = torch.cuda.current_stream(device)
    st.wait_stream(caller)   # the tile's points
    s = st.cuda_stream
    with torch.cuda.stream(st):
        t = _abi.cg_tile(d_tile_ptr, first, n, n_total, point_step, *offsets)
        keys = torch.empty(_abi.CG_TILE_KEYS, dtype=torch.int32, device=device)
        _abi.check(lib.cg_tile_front_async(h, C.byref(t), keys.data_ptr(), s))
        merged = merge_tile_keys_dev(keys, device)
        counts = torch.empty(_abi.CG_TILE_COUNTS, dtype=torch.int32, device=device)
        _abi.check(lib.cg_tile_decide_async(h, merged.data_ptr(), counts.data_ptr(), s))
        if not _distributed():
            if order is None:
                _abi.check(lib.cg_tile_backend_own(h, n_total, s))
            else:   # (the voxel order is read when the backend's launches are enqueued)
                prev = engine.voxel_order
                engine.set_voxel_order(order)
                try:
                    _abi.check(lib.cg_tile_backend_own(h, n_total, s))
                finally:
                    engine.set_voxel_order(prev)
            # the caller's stream waits for the frame: its tile buffer and the handle's
            # outputs are safe to reuse or read there once this returns (fetch=False)
            caller.wait_stream(st)
            return engine.fetch(0) if fetch else True
        total, sizes = merge_tile_counts_dev(counts, device)
        ns = sizes[dist.get_rank()]
        sp = torch.empty((max(ns, 1), 4), dtype=torch.float32, device=device)
        si = torch.empty((max(ns, 1),), dtype=torch.int32, device=device)
        _abi.check(lib.cg_tile_survivors_async(h, sp.data_ptr(), si.data_ptr(), ns, s))
        gp, gi = gather_survivors(sp[:ns], si[:ns], device, dst, sizes=sizes)
        if dist.get_rank() != dst:
            return None
        st.synchronize()   # cg_tile_backend runs on the handle's own stream
    _abi.check(lib.cg_tile_backend(h, gp.data_ptr(), gi.data_ptr(), int(gp.shape[0]), total.ctypes.data, n_total))
    return engine.fetch(0) if fetch else True


# ---------------------------------------------------------------------------------------------
# C5 backend tiled by voxel slabs with a halo exchange (include/cones_gpu.h, cg_halo_*).
# Collectives per frame after the survivors are known: one all-to-all of the slab counts and
# one of the survivors (each to its slab's rank), one all-gather of the record counts, one
# point-to-point halo (each slab's lowest `band` voxel columns to the slab below), one
# all-gather of the pair counts and one gather of the records and pairs to dst.

def _split_exchange(rows, dest, world_size, device):
    """rows (n, k) float32 with dest (n,) int32 in [-1, world): rows go to rank dest (in their
    order; -1 dropped). Returns the rows this rank receives, in source-rank order."""
    cd = _coll_device(device)
    keep = dest >= 0
    order = torch.argsort(dest[keep].to(torch.int64), stable=True)
    send = rows[keep][order].to(cd).contiguous()
    cnt = torch.bincount(dest[keep].to(torch.int64), minlength=world_size).to(cd)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt)
    rc, sc = torch.stack([rcnt, cnt]).cpu().tolist()   # the one host read: both split lists
    out = torch.empty((sum(rc), rows.shape[1]), dtype=rows.dtype, device=cd)
    dist.all_to_all_single(out, send, rc, sc)
    return out.to(device)


def _all_gather_ints(vals, device):
    cd = _coll_device(device)
    t = torch.tensor(vals, dtype=torch.int64, device=cd)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return torch.stack(parts).cpu().tolist()


last_halo_stats = {}   # the rank's figures of its last run_halo_backend call (tests, bench)


def _torch_done(device):
    """The cg_halo_* calls run on the handle's own stream, which nothing orders after torch's
    current stream: the tensors they read (gathered, exchanged, sliced there) must be complete
    first. Every cg_halo_* call returns with its reads done (each ends in a stream wait, and the
    one-slab cg_halo_local copies its survivors and then waits), so the caller may free or reuse
    those tensors afterwards."""
    torch.cuda.current_stream(device).synchronize()


def run_halo_backend(engine, total, sp, si, n_total: int, device, dst: int = 0, fetch: bool = True, sizes=None):
    """The backend of a tiled frame from every rank's survivors (sp (ns, 4) float32, si (ns,)
    frame indices) and the merged counts: slab voxelisation and clustering, halo edges, merge on
    dst. Returns the Detection on dst, None elsewhere, or False when the frame has no voxel
    lattice (PCL's overflow guard) and the caller must gather instead. `sizes`: every rank's
    survivor count (the one-slab case gathers the survivors to dst)."""
    import ctypes as C
    from . import _abi
    lib, h = _abi.lib(), engine.handle
    ws = dist.get_world_size() if _distributed() else 1
    rank = dist.get_rank() if _distributed() else 0
    plan = _abi.cg_halo_plan()
    _abi.check(lib.cg_halo_plan_frame(h, total.ctypes.data, n_total, ws, C.byref(plan)))
    if plan.passthrough:
        return False
    ns = int(sp.shape[0])
    if plan.slabs == 1:
        # one slab has no boundary: its backend is the frame's, so cg_halo_local takes every
        # survivor (on dst) and writes the results itself, asynchronously; no records, no merge
        last_halo_stats.clear()   # voxels: None on dst (on the device), 0 elsewhere
        last_halo_stats.update(slabs=1, slab_w=int(plan.slab_w), band=int(plan.band), survivors=ns,
                               voxels=None if rank == dst else 0, halo_sent=0, halo_received=0, pairs=0,
                               path="run_halo_backend: one slab (cg_halo_plan_frame, survivor gather, "
                                    "cg_halo_local)")
        if _distributed():
            sp, si = gather_survivors(sp, si, device, dst, sizes=sizes)
            if rank != dst:
                return None
            ns = int(sp.shape[0])
        nv = C.c_uint32(0)
        _torch_done(device)
        _abi.check(lib.cg_halo_local(h, C.byref(plan), sp.data_ptr(), si.data_ptr(), ns, plan.n_pads,
                                     total.ctypes.data, n_total, None, 0, C.byref(nv)))
        return engine.fetch(0) if fetch else True
    slab = torch.empty((max(ns, 1),), dtype=torch.int32, device=device)
    _torch_done(device)
    _abi.check(lib.cg_halo_owner(h, C.byref(plan), sp.data_ptr(), ns, slab.data_ptr()))
    slab = slab[:ns]
    # survivors to their slab's rank; sources hold ascending frame-index ranges, so every rank
    # receives its slab's survivors in frame-index order
    if _distributed():
        rows = torch.cat([sp, si.view(torch.float32).unsqueeze(1)], 1)
        got = _split_exchange(rows, slab, ws, device)
        mp_, mi = got[:, :4].contiguous(), got[:, 4].contiguous().view(torch.int32)
    else:
        keep = slab >= 0
        mp_, mi = sp[keep].contiguous(), si[keep].contiguous()
    n = int(mp_.shape[0])
    npad = plan.n_pads if rank == plan.pad_slab else 0
    cap = n + npad
    rec = torch.empty((max(cap, 1), _abi.CG_HALO_REC_WORDS), dtype=torch.int32, device=device)
    nv = C.c_uint32(0)
    _torch_done(device)
    _abi.check(lib.cg_halo_local(h, C.byref(plan), mp_.data_ptr(), mi.data_ptr(), n, npad, total.ctypes.data,
                                 n_total, rec.data_ptr(), rec.shape[0], C.byref(nv)))
    rec = rec[: nv.value]
    col = rec[:, 4] % int(plan.div_b[0])
    lo = rank * plan.slab_w
    top = rec[col >= lo + plan.slab_w - plan.band].contiguous()    # own side of the upper edge
    low = rec[col < lo + plan.band].contiguous()                   # halo for the slab below
    halo = torch.empty((0, _abi.CG_HALO_REC_WORDS), dtype=torch.int32, device=device)
    if _distributed():
        counts = _all_gather_ints([int(rec.shape[0]), int(low.shape[0])], device)
        cd = _coll_device(device)
        ops = []
        if 0 < rank < plan.slabs and low.shape[0]:
            ops.append(dist.P2POp(dist.isend, low.to(cd), rank - 1))
        nh = counts[rank + 1][1] if rank + 1 < min(ws, plan.slabs) else 0
        if nh:
            hbuf = torch.empty((nh, _abi.CG_HALO_REC_WORDS), dtype=torch.int32, device=cd)
            ops.append(dist.P2POp(dist.irecv, hbuf, rank + 1))
        if ops:
            for q in dist.batch_isend_irecv(ops):
                q.wait()
        if nh:
            halo = hbuf.to(device)
    pairs = torch.empty((max(4 * halo.shape[0], 64), 2), dtype=torch.int32, device=device)
    npairs = C.c_uint32(0)
    for _ in range(2 if halo.shape[0] and top.shape[0] else 0):   # no halo rows (the top slab, one rank): no edges
        _torch_done(device)
        _abi.check(lib.cg_halo_edges(h, top.data_ptr(), top.shape[0], halo.data_ptr(), halo.shape[0],
                                     pairs.data_ptr(), pairs.shape[0], C.byref(npairs)))
        if npairs.value <= pairs.shape[0]:   # once more with room for every pair when the first guess was short
            break
        pairs = torch.empty((npairs.value, 2), dtype=torch.int32, device=device)
    pairs = pairs[: npairs.value]
    last_halo_stats.clear()
    last_halo_stats.update(slabs=int(plan.slabs), slab_w=int(plan.slab_w), band=int(plan.band), survivors=n,
                           voxels=int(rec.shape[0]), halo_sent=int(low.shape[0]) if 0 < rank < plan.slabs else 0,
                           halo_received=int(halo.shape[0]), pairs=int(pairs.shape[0]),
                           path="run_halo_backend: voxel slabs (all-to-all, cg_halo_local, P2P halo, "
                                "cg_halo_edges, gather, cg_halo_merge)")
    if _distributed():
        sizes = _all_gather_ints([int(rec.shape[0]), int(pairs.shape[0])], device)
        vmax = max(1, max(s[0] for s in sizes))
        pmax = max(1, max(s[1] for s in sizes))
        cd = _coll_device(device)
        W = _abi.CG_HALO_REC_WORDS
        pack = torch.zeros((vmax * W + pmax * 2,), dtype=torch.int32, device=cd)
        pack[: rec.numel()] = rec.reshape(-1).to(cd)
        pack[vmax * W: vmax * W + pairs.numel()] = pairs.reshape(-1).to(cd)
        bufs = [torch.empty_like(pack) for _ in range(ws)] if rank == dst else None
        dist.gather(pack, bufs, dst=dst)
        if rank != dst:
            return None
        rec = torch.cat([bufs[r][: sizes[r][0] * W].view(-1, W) for r in range(ws)], 0).to(device)
        pairs = torch.cat([bufs[r][vmax * W: vmax * W + sizes[r][1] * 2].view(-1, 2) for r in range(ws)],
                          0).to(device)
    rec, pairs = rec.contiguous(), pairs.contiguous()
    _torch_done(device)
    _abi.check(lib.cg_halo_merge(h, C.byref(plan), rec.data_ptr(), rec.shape[0], pairs.data_ptr(), pairs.shape[0],
                                 total.ctypes.data, n_total))
    return engine.fetch(0) if fetch else True
