"""C5 tiling end to end on the GPU: one frame split into contiguous point tiles over ranks
(torch.distributed, gloo here so that 2-3 ranks can share the box's single GPU; RCCL on a
multi-GPU node), merged with the cg_tile_* protocol, backend on rank 0. The result must be
bit-identical to the CPU restatement on the whole frame."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import cones_perception_amd as cp
import oracle_py as O
from cones_perception_amd import Detection
from helpers import assert_same_detection, assert_same_cluster_sets

pytestmark = pytest.mark.gpu

FIELDS = ("n_points", "n_kept", "n_filtered", "voxels", "labels", "cluster_offsets", "cluster_indices",
          "centroids", "flags")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frame(rings, cols, mutate=None):
    raw = cp.synth_frames(1, first_frame=4, rings=rings, cols=cols, clutter=40, cones_per_row=10)
    pts = raw[0].view(np.float32).reshape(-1, 4)
    if mutate == "passthrough":       # a few points 1 km up: PCL's int32 voxel-count guard trips
        pts[5::20011, 2] = 1000.0
    elif mutate == "narrow":          # x squeezed to a few voxel columns: fewer slabs than ranks
        pts[:, 0] *= np.float32(0.01)
    elif mutate == "nonfinite":       # NaN / inf survivors are not voxelised
        pts[7::9973, 0] = np.nan
        pts[11::7919, 1] = np.inf
    return raw


def _worker(rank, world, port, out, rings, cols, over, halo=False, mutate=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cones_perception_amd as cpp
    from cones_perception_amd import dist as cd
    params = cpp.load_params("simulation", over)
    raw = _frame(rings, cols, mutate)
    n_total = rings * cols
    lo, hi = cd.tile_range(n_total, rank, world)
    dev = torch.device("cuda", 0)
    tile = torch.from_numpy(np.ascontiguousarray(raw[0, lo * 16: hi * 16])).to(dev)
    eng = cpp.BatchEngine(params, device=0)
    det = cd.run_tiled_frame(eng, tile.data_ptr(), lo, hi - lo, n_total, dev, halo=halo)
    st = [dict(cd.last_halo_stats)]
    if halo and dist.get_world_size() > 1:
        allst = [None] * world
        dist.all_gather_object(allst, st[0])
        st = allst
    if rank == 0:
        np.savez(out, stats=np.array(json.dumps(st)), **{k: np.asarray(getattr(det, k)) for k in FIELDS})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rings,cols,over,halo,mutate", [
    (2, 128, 2048, {}, False, None),
    (3, 96, 2048, {}, False, None),
    (2, 64, 2048, {"distance_treshold_min": 0.0}, False, None),   # zero pads survive: global backend on rank 0
    # voxel slabs with a halo exchange: clusters cross slab edges, pads on one slab
    (2, 128, 2048, {}, True, None),
    (3, 96, 2048, {}, True, None),
    (4, 64, 2048, {"distance_treshold_min": 0.0}, True, None),
    (4, 64, 2048, {"distance_treshold_max": 30.0, "max_cluster_size": 100000}, True, None),   # the wall: long clusters
    (3, 64, 2048, {"distance_treshold_max": 1e5}, True, "passthrough"),   # no lattice: falls back to the gather
    (3, 64, 2048, {}, True, "narrow"),
    (2, 64, 2048, {}, True, "nonfinite"),
    # C5's own frame size: 1,048,576 points over 2 ranks, both forms
    (2, 128, 8192, {}, False, None),
    (2, 128, 8192, {}, True, None),
])
def test_tiled_frame_matches_oracle(tmp_path, world, rings, cols, over, halo, mutate):
    out = str(tmp_path / "r0.npz")
    mp.spawn(_worker, args=(world, _free_port(), out, rings, cols, over, halo, mutate), nprocs=world, join=True)
    z = np.load(out)
    got = Detection(*(z[k].item() if z[k].ndim == 0 else z[k] for k in FIELDS))
    params = cp.load_params("simulation", over)
    raw = _frame(rings, cols, mutate)
    # the halo form sums each voxel in frame-index order on its slab (ORDER_STABLE); the gather
    # form runs the global backend, which reproduces PCL's std::sort order
    ref, _ = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE, O.ORDER_STABLE if halo else O.ORDER_PCL)
    assert got.n_points == rings * cols
    assert_same_detection(got, ref, f"tiled x{world} halo={halo}")
    if halo:   # the north star's bar against PCL's own voxel order: same cluster sets, centroids within 1e-5 m
        pcl, _ = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE, O.ORDER_PCL)
        assert_same_cluster_sets(got, pcl, f"tiled x{world} halo vs ORDER_PCL")
    if mutate == "passthrough":
        assert got.flags & 1                                    # PCL's guard: voxel cloud = input
    if halo and mutate != "passthrough":
        # the halo path ran on every slab; the wall case's clusters cross every slab edge
        st = json.loads(str(z["stats"]))
        if mutate == "narrow":
            assert all(s["slabs"] < world for s in st) and st[-1]["voxels"] == 0, st
            return
        assert all(s["slabs"] == world for s in st), st
        assert sum(s["voxels"] for s in st) == got.voxels.shape[0], st
        assert all(s["halo_received"] > 0 for s in st[:-1]), st
        if "max_cluster_size" in over:
            assert all(s["pairs"] > 0 for s in st[:-1]), st


@pytest.mark.parametrize("halo", [False, True])
def test_tiled_single_rank_matches_oracle(halo):
    """World size 1 (no process group): the tile protocol on one tile = the whole frame."""
    import torch
    from cones_perception_amd import dist as cd
    params = cp.load_params("simulation")
    raw = cp.synth_frames(1, first_frame=9, rings=80, cols=1024, clutter=40, cones_per_row=8)
    n = raw.shape[1] // 16
    d = torch.from_numpy(raw[0].copy()).to(torch.device("cuda", 0))
    got = cd.run_tiled_frame(cp.BatchEngine(params, device=0), d.data_ptr(), 0, n, n, torch.device("cuda", 0),
                             halo=halo)
    ref, _ = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE, O.ORDER_STABLE if halo else O.ORDER_PCL)
    assert_same_detection(got, ref, "tiled x1")
    if halo:
        pcl, _ = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE, O.ORDER_PCL)
        assert_same_cluster_sets(got, pcl, "tiled x1 halo vs ORDER_PCL")


def test_tile_async_argument_checks():
    """The async tile entry points refuse calls out of order and tiles that do not fit the
    call: no kernel is launched for a refused call, and the handle stays usable."""
    import ctypes as C
    import torch
    from cones_perception_amd import _abi
    lib = _abi.lib()
    dev = torch.device("cuda", 0)
    eng = cp.BatchEngine(cp.load_params("simulation"), device=0)
    h = eng.handle
    raw = cp.synth_frames(1, first_frame=3, rings=16, cols=1024, clutter=10, cones_per_row=4)
    n = raw.shape[1] // 16
    d = torch.from_numpy(raw[0].copy()).to(dev)
    keys = torch.empty(_abi.CG_TILE_KEYS, dtype=torch.int32, device=dev)
    counts = torch.empty(_abi.CG_TILE_COUNTS, dtype=torch.int32, device=dev)
    sp = torch.empty(n * 4, dtype=torch.float32, device=dev)
    si = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    # before any cg_tile_front_async
    assert lib.cg_tile_decide_async(h, keys.data_ptr(), counts.data_ptr(), s) == _abi.CG_E_INVALID
    assert lib.cg_tile_survivors_async(h, sp.data_ptr(), si.data_ptr(), 0, s) == _abi.CG_E_INVALID
    assert lib.cg_tile_backend_own(h, n, s) == _abi.CG_E_INVALID
    # a tile running past the end of its frame, a null tile pointer
    bad = _abi.cg_tile(d.data_ptr(), n // 2, n, n, 16, 0, 4, 8, 12)
    assert lib.cg_tile_front_async(h, C.byref(bad), keys.data_ptr(), s) == _abi.CG_E_INVALID
    assert lib.cg_tile_front_async(h, C.byref(_abi.cg_tile(0, 0, n, n, 16, 0, 4, 8, 12)), keys.data_ptr(),
                                   s) == _abi.CG_E_INVALID
    # the first half of a frame: the backend needs the whole frame in the tile
    half = n // 2
    t = _abi.cg_tile(d.data_ptr(), 0, half, n, 16, 0, 4, 8, 12)
    _abi.check(lib.cg_tile_front_async(h, C.byref(t), keys.data_ptr(), s))
    _abi.check(lib.cg_tile_decide_async(h, keys.data_ptr(), counts.data_ptr(), s))
    assert lib.cg_tile_backend_own(h, n, s) == _abi.CG_E_INVALID
    assert lib.cg_tile_survivors_async(h, sp.data_ptr(), si.data_ptr(), half + 1, s) == _abi.CG_E_INVALID
    assert lib.cg_tile_survivors_async(h, 0, 0, 1, s) == _abi.CG_E_INVALID
    torch.cuda.synchronize(dev)
    # the handle still runs a whole frame through the tile protocol, bit-exact
    from cones_perception_amd import dist as cd
    params = cp.load_params("simulation")
    got = cd.run_tiled_frame(eng, d.data_ptr(), 0, n, n, dev)
    ref, _ = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE, O.ORDER_PCL)
    assert_same_detection(got, ref, "tiled after refused calls")
