"""C4 on the HIP engine with several ranks: the root scatters the frame batch
(dist.scatter_frames), every rank runs its share through the batch engine (cg_run_batch on
the GPU), and the per-frame result headers come back to the root (dist.gather_headers).

Two gloo ranks share the box's one GPU (RCCL needs one GPU per rank; tests/test_gpu_rccl.py
runs the same composition under RCCL at world size 1). The root checks every gathered header
against the CPU restatement on the whole batch, and every rank checks each of its frames'
fetched results bit for bit (voxels, labels, cluster sets, centroids) against it.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import cones_perception_amd as cp
import oracle_py as O

pytestmark = pytest.mark.gpu

F, RINGS, COLS = 32, 64, 1024   # 32 frames of 65,536 points per rank


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _header_row(det):
    return [det.n_points, det.n_kept, det.n_filtered, len(det.voxels), len(det.centroids), det.flags, 0, 0]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cones_perception_amd as cpp
    from cones_perception_amd import dist as cd
    from helpers import assert_same_detection
    params = cpp.load_params("simulation")
    n = RINGS * COLS
    allf = torch.from_numpy(cpp.synth_frames(F * world, first_frame=0, rings=RINGS, cols=COLS)) if rank == 0 else None
    mine = cd.scatter_frames(allf, F, n * 16, torch.device("cpu"))   # (gloo: host tensors)
    d = mine.to(torch.device("cuda", 0))
    eng = cpp.BatchEngine(params, device=0)
    eng.run(d.data_ptr(), F, n, 16)
    rows, exact = [], 0
    mine_np = mine.numpy()
    for i in range(F):
        det = eng.fetch(i)
        rows.append(_header_row(det))
        ref, _ = O.run(params, cpp.frame_cloud(mine_np[i]), O.MODE_PIPELINE)
        assert_same_detection(det, ref, f"rank {rank} frame {i}")
        exact += 1
    hdr = cd.gather_headers(torch.tensor(rows, dtype=torch.int32))
    counts = torch.tensor([exact], dtype=torch.int64)
    allc = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(allc, counts)
    if rank == 0:
        np.savez(out, hdr=hdr.numpy(), exact=torch.cat(allc).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_c4_scatter_batch_gather_matches_oracle(tmp_path, world):
    out = str(tmp_path / "c4.npz")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    z = np.load(out)
    assert z["exact"].tolist() == [F] * world   # every rank: every frame bit-exact
    params = cp.load_params("simulation")
    raw = cp.synth_frames(F * world, first_frame=0, rings=RINGS, cols=COLS)
    want = []
    for i in range(F * world):
        ref, _ = O.run(params, cp.frame_cloud(raw[i]), O.MODE_PIPELINE)
        want.append(_header_row(ref))
    assert np.array_equal(z["hdr"], np.array(want, np.int32))
