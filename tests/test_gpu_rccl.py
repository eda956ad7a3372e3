"""The multi-GPU code paths under RCCL ("nccl") on the box's one GPU: a world-size-1 process
group with collectives forced on (dist.force_collectives), so that every device-tensor
collective the 8-GPU driver run uses executes under RCCL here first (the C4
scatter/gather is rccl.h's ncclScatter / ncclGather). One rank only: RCCL refuses two ranks
on one device, and gloo (tests/test_gpu_tiled.py) routes collectives through host tensors.

Every check runs in one spawned process (the process group must not outlive the test); a
failing assertion there fails the test with its traceback."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    from cones_perception_amd import dist as cd
    cd.force_collectives(True)
    assert cd._distributed()
    return torch, dist, cd


def _c4_worker(rank, port, frames):
    torch, dist, cd = _init(port)
    import cones_perception_amd as cp
    import oracle_py as O
    from helpers import assert_same_detection
    dev = torch.device("cuda", 0)
    params = cp.load_params("simulation")
    raw = cp.synth_frames(frames, first_frame=0, rings=64, cols=1024, threads=8)
    allf = torch.from_numpy(raw).to(dev)
    mine = cd.scatter_frames(allf, frames, raw.shape[1], dev)      # RCCL scatter from rank 0
    torch.cuda.synchronize(dev)
    assert mine.is_cuda and torch.equal(mine, allf)
    eng = cp.BatchEngine(params, device=0)
    st = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    eng.run(mine.data_ptr(), frames, 65536, 16, stream=st.cuda_stream)
    torch.cuda.current_stream(dev).wait_stream(st)
    hdr = torch.empty((frames, 8), dtype=torch.int32, device=dev)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyDtoDAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    assert hip.hipMemcpyDtoDAsync(hdr.data_ptr(), eng.results().d_header, frames * 32,
                                  ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) == 0
    got = cd.gather_headers(hdr)                                   # RCCL gather to rank 0
    torch.cuda.synchronize(dev)
    got = got.cpu().numpy()
    assert got.shape == (frames, 8)
    for i in range(frames):
        det = eng.fetch(i)
        ref, _ = O.run(params, cp.frame_cloud(raw[i]), O.MODE_PIPELINE, O.ORDER_PCL)
        assert_same_detection(det, ref, f"C4 frame {i}")
        assert got[i, 0] == 65536 and got[i, 1] == det.n_kept and got[i, 2] == det.n_filtered
        assert got[i, 3] == det.voxels.shape[0] and got[i, 4] == det.centroids.shape[0], (i, got[i])
    t = cd.max_over_ranks(3.5, dev)
    assert t == 3.5
    dist.destroy_process_group()


def _collectives_worker(rank, port):
    torch, dist, cd = _init(port)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    for it in range(8):
        keys = rng.integers(0, 2 ** 32, 19, dtype=np.uint64).astype(np.uint32)
        keys[18] = rng.integers(0, 2 ** 18, dtype=np.uint64)
        dk = torch.from_numpy(keys.view(np.int32).copy()).to(dev)
        mk = cd.merge_tile_keys_dev(dk, dev)                       # int64 MIN all-reduce on the GPU
        assert mk.is_cuda
        assert np.array_equal(mk.cpu().numpy().view(np.uint32), keys), it
        hk = cd.merge_tile_keys(keys, dev)                         # host-array form, same collective
        assert np.array_equal(hk, keys), it
        counts = rng.integers(0, 2 ** 32, 9, dtype=np.uint64).astype(np.uint32)
        counts[:3] = rng.integers(0, 1 << 20, 3, dtype=np.uint64)
        tot, sizes = cd.merge_tile_counts_dev(torch.from_numpy(counts.view(np.int32).copy()).to(dev), dev)
        assert np.array_equal(tot, counts) and sizes == [int(counts[1])], it
        htot, hsz = cd.merge_tile_counts(counts, dev, per_rank=True)
        assert np.array_equal(htot, counts) and hsz == [int(counts[1])], it
    # survivors: (n, 4) points and frame indices, gathered with the index bit-cast as a column
    for n in (0, 1, 777):
        p = torch.from_numpy(rng.standard_normal((n, 4)).astype(np.float32)).to(dev)
        i = torch.from_numpy(rng.integers(0, 2 ** 31, n).astype(np.int32)).to(dev)
        gp, gi = cd.gather_survivors(p, i, dev, sizes=[n])
        assert gp.is_cuda and torch.equal(gp, p) and torch.equal(gi, i), n
        gp, gi = cd.gather_survivors(p, i, dev)                    # sizes all-gathered first
        assert torch.equal(gp, p) and torch.equal(gi, i), n
    # the halo form's uneven all-to-all: rows with dest -1 are dropped, the others arrive in order
    for n in (0, 5, 1000):
        rows = torch.from_numpy(rng.standard_normal((n, 5)).astype(np.float32)).to(dev)
        dest = torch.from_numpy(rng.integers(-1, 1, n).astype(np.int32)).to(dev)
        got = cd._split_exchange(rows, dest, 1, dev)
        assert got.is_cuda and torch.equal(got, rows[dest >= 0]), n
    allneg = torch.full((9,), -1, dtype=torch.int32, device=dev)
    got = cd._split_exchange(torch.ones((9, 5), device=dev), allneg, 1, dev)
    assert got.shape == (0, 5)
    dist.destroy_process_group()


def _tiled_worker(rank, port, halo):
    torch, dist, cd = _init(port)
    import cones_perception_amd as cp
    import oracle_py as O
    from helpers import assert_same_detection, assert_same_cluster_sets
    dev = torch.device("cuda", 0)
    params = cp.load_params("simulation")
    raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
    n = raw.shape[1] // 16
    tile = torch.from_numpy(raw[0].copy()).to(dev)
    eng = cp.BatchEngine(params, device=0)
    det = cd.run_tiled_frame(eng, tile.data_ptr(), 0, n, n, dev, halo=halo)
    ref, _ = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE, O.ORDER_PCL)
    if halo:   # voxel sums in frame-index order on each slab: the north star's bar against PCL's order
        st, _ = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE, O.ORDER_STABLE)
        assert_same_detection(det, st, "tiled halo x1 (nccl), point order")
        assert_same_cluster_sets(det, ref, "tiled halo x1 (nccl) vs PCL order")
    else:
        assert_same_detection(det, ref, "tiled gather x1 (nccl)")
    dist.destroy_process_group()


def test_rccl_c4_scatter_batch_gather():
    """C4 under RCCL: rank 0 scatters 256 x 64k frames, the batch engine runs them, per-frame
    headers gathered back; every frame bit-exact against the oracle (PCL voxel order)."""
    mp.spawn(_c4_worker, args=(_free_port(), 256), nprocs=1, join=True)


def test_rccl_tile_collectives_on_device_tensors():
    """merge_tile_keys(_dev), merge_tile_counts(_dev), gather_survivors, _split_exchange on
    device tensors under RCCL, including empty inputs and dropped rows."""
    mp.spawn(_collectives_worker, args=(_free_port(),), nprocs=1, join=True)


@pytest.mark.parametrize("halo", [False, True])
def test_rccl_tiled_c5_frame(halo):
    """The tiled C5 protocol on the 1,048,576-point frame with every collective under RCCL."""
    mp.spawn(_tiled_worker, args=(_free_port(), halo), nprocs=1, join=True)
