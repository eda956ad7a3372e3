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
