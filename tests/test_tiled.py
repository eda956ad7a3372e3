"""C5 tiling helpers (cones_perception_amd.dist): merge rules and the survivor gather, with
world-size-2 gloo on CPU (no GPU). The GPU end-to-end check is tests/test_gpu_tiled.py."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cones_perception_amd import dist as cd


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    keys = np.arange(19, dtype=np.uint32) * 10 + rank          # rank 0 holds the minima
    keys[5] = 1000 - rank                                         # rank 1 holds this one
    keys[18] = (1 << rank) | (1 << 17)                            # used-bin masks
    mk = cd.merge_tile_keys(keys, dev)
    counts = np.array([100 + rank, 10 * (rank + 1), 7, 50 - rank, 60, 70 + rank, 80, 90 - rank, 95], np.uint32)
    mc = cd.merge_tile_counts(counts, dev)
    n = 3 + 2 * rank
    pts = torch.full((n, 4), float(rank))
    idx = torch.arange(n, dtype=torch.int32) + 1000 * rank
    gp, gi = cd.gather_survivors(pts, idx, dev)
    # the single-gather form run_tiled_frame uses: sizes from the count words
    counts[1] = n
    mc2, sizes = cd.merge_tile_counts(counts, dev, per_rank=True)
    gp2, gi2 = cd.gather_survivors(pts, idx, dev, sizes=sizes)
    idx[0] = -7                                                   # negative indices survive the bit-cast
    gp3, gi3 = cd.gather_survivors(pts, idx, dev, sizes=sizes)
    z = np.zeros(0)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), mk=mk, mc=mc, sizes=np.array(sizes),
             gp=gp.numpy() if gp is not None else z, gi=gi.numpy() if gi is not None else z,
             gp2=gp2.numpy() if gp2 is not None else z, gi2=gi2.numpy() if gi2 is not None else z,
             gi3=gi3.numpy() if gi3 is not None else z)
    dist.destroy_process_group()


def test_tile_merges_and_gather(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = np.load(tmp_path / "r0.npz"), np.load(tmp_path / "r1.npz")
    for r in (r0, r1):                       # every rank sees the same merged words
        want = np.arange(19, dtype=np.uint32) * 10
        want[5] = 999
        assert np.array_equal(r["mk"][:18], want[:18])
        assert r["mk"][18] == (1 | 2 | (1 << 17))
        assert list(r["mc"]) == [201, 30, 14, 49, 60, 70, 80, 90, 95]
    assert r0["gp"].shape == (3 + 5, 4) and r1["gp"].size == 0
    assert list(r0["gi"]) == [0, 1, 2, 1000, 1001, 1002, 1003, 1004]
    assert np.array_equal(r0["gp"][:3], np.zeros((3, 4))) and np.array_equal(r0["gp"][3:], np.ones((5, 4)))
    assert list(r0["sizes"]) == [3, 5] and list(r1["sizes"]) == [3, 5]
    assert np.array_equal(r0["gp2"], r0["gp"]) and np.array_equal(r0["gi2"], r0["gi"])
    assert r0["gi2"].dtype == np.int32 and r1["gp2"].size == 0
    assert list(r0["gi3"]) == [-7, 1, 2, -7, 1001, 1002, 1003, 1004]


def test_tile_ranges_cover_the_frame():
    for n, w in ((1048576, 8), (1000, 3), (5, 8)):
        rs = [cd.tile_range(n, r, w) for r in range(w)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))


def _split_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(rank)
    n = 5 + 4 * rank
    idx = torch.arange(n, dtype=torch.int32) + 100 * rank            # ascending frame indices
    dest = torch.randint(-1, world, (n,), generator=g, dtype=torch.int32)
    rows = torch.cat([idx.to(torch.float32).unsqueeze(1), dest.to(torch.float32).unsqueeze(1)], 1)
    got = cd._split_exchange(rows, dest, world, torch.device("cpu"))
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), idx=idx.numpy(), dest=dest.numpy(), got=got.numpy())
    dist.destroy_process_group()


def test_split_exchange_delivers_in_frame_index_order(tmp_path):
    """The halo path's all-to-all (run_halo_backend): every rank receives exactly the rows
    addressed to it, in source-rank then source order (= frame-index order), -1 dropped."""
    world = 3
    mp.spawn(_split_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    zs = [np.load(tmp_path / f"s{r}.npz") for r in range(world)]
    idx = np.concatenate([z["idx"] for z in zs])
    dest = np.concatenate([z["dest"] for z in zs])
    for r in range(world):
        want = idx[dest == r]
        got = zs[r]["got"]
        assert np.array_equal(got[:, 0].astype(np.int64), want)
        assert np.all(got[:, 1] == r)


def test_halo_slab_decomposition_restates_global_clusters():
    """The halo algorithm in numpy (design check, no GPU): voxel columns cut into slabs of at
    least `band` columns (the plan's arithmetic); components per slab; only the records of a
    slab's lowest `band` columns cross to the slab below, joined against its top `band`
    columns; uniting the slab components along those pairs gives the global components of
    the whole voxel cloud, for 1-8 slabs."""
    import sys
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import cones_perception_amd as cp
    import np_reference as R
    prm = {"voxel_filter_leaf_size_x": 0.04, "voxel_filter_leaf_size_y": 0.04, "voxel_filter_leaf_size_z": 0.04}
    F32 = np.float32
    raw = cp.synth_frames(1, first_frame=3, rings=32, cols=1024, clutter=20, cones_per_row=6)
    pts = np.frombuffer(raw[0].tobytes(), F32).reshape(-1, 4)
    d2 = (pts[:, 0].astype(np.float64) ** 2 + pts[:, 1] ** 2 + pts[:, 2] ** 2)
    pts = pts[(d2 < 12.0 ** 2) & (pts[:, 2] > -0.45)]                  # a cone field without the ground
    vox, passthrough = R.voxel_grid(pts, prm)
    assert not passthrough and vox.shape[0] > 100
    inv = F32(25.0)
    col = (np.floor(vox[:, 0] * inv) - np.floor(pts[:, 0].min() * inv)).astype(np.int64)
    tol = F32(np.sqrt(np.float64(F32(0.325)) ** 2 + np.float64(F32(0.228)) ** 2))
    r2 = F32(np.float64(tol) * np.float64(tol))
    band = int(np.ceil(np.float64(np.sqrt(np.float64(r2))) * 25.0)) + 2
    p = vox[:, :3]

    def adjacent(a, b):
        d = p[a][:, None, :] - p[b][None, :, :]
        return ((d[..., 0] * d[..., 0]) + (d[..., 1] * d[..., 1])) + (d[..., 2] * d[..., 2]) < r2

    def components(ids):
        a = adjacent(ids, ids)
        ii, jj = np.nonzero(a)
        _, lab = connected_components(coo_matrix((np.ones(ii.size), (ii, jj)), shape=(ids.size, ids.size)),
                                      directed=False)
        root = {}
        for k, l in enumerate(lab):
            root.setdefault(l, ids[k])                                  # lowest voxel of each component
        return {ids[k]: root[l] for k, l in enumerate(lab)}

    V = vox.shape[0]
    full = components(np.arange(V))
    div_x = int(col.max()) + 1
    crossed = 0
    for world in range(1, 9):
        slabs = max(1, min(world, div_x // band))
        w = -(-div_x // slabs)
        slab = np.minimum(col // w, slabs - 1)
        comp = {}
        for s in range(slabs):
            comp.update(components(np.nonzero(slab == s)[0]))
        par = {v: comp[v] for v in range(V)}

        def find(x):
            while par[x] != x:
                x = par[x]
            return x
        for s in range(slabs - 1):
            top = np.nonzero((slab == s) & (col >= (s + 1) * w - band))[0]
            low = np.nonzero((slab == s + 1) & (col < (s + 1) * w + band))[0]
            if top.size and low.size:
                for a, b in zip(*np.nonzero(adjacent(top, low))):
                    ra, rb = find(comp[top[a]]), find(comp[low[b]])
                    if ra != rb:
                        par[max(ra, rb)] = min(ra, rb)
                        crossed += 1
        assert all(find(v) == full[v] for v in range(V)), f"{world} slabs"
    assert crossed > 0                                                  # components did cross slab edges
