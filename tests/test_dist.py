"""World-size-2 gloo runs of the multi-GPU plumbing (cones_perception_amd/dist.py) on CPU:
frame ownership, max-over-ranks timing, root scatter of frames and gather of per-frame result
headers. Per-frame results come from the CPU restatement (the GPU path needs a device), so
this checks that sharded processing + gather equals processing the whole batch in one rank."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F, RINGS, COLS = 3, 16, 256


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _headers(frames):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cones_perception_amd as cp
    import oracle_py as O
    params = cp.load_params("simulation")
    out = np.zeros((frames.shape[0], 8), np.int32)
    for i in range(frames.shape[0]):
        det, hdr = O.run(params, cp.frame_cloud(frames[i]), O.MODE_PIPELINE)
        out[i, :5] = hdr[:5].astype(np.int32)
        out[i, 5] = int(np.abs(det.centroids).sum() * 1000) if len(det.centroids) else 0
    return out


def _worker(rank, ws, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import cones_perception_amd as cp
    from cones_perception_amd import dist as cd
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    dev = torch.device("cpu")
    # (1) weak-scaling ownership: each rank synthesises its own frames
    mine = list(cd.frame_range(rank, F))
    own = cp.synth_frames(F, first_frame=mine[0], rings=RINGS, cols=COLS)
    # (2) C4 composition: root scatters the whole batch; must equal the owned frames
    allf = torch.from_numpy(cp.synth_frames(F * ws, first_frame=0, rings=RINGS, cols=COLS)) if rank == 0 else None
    got = cd.scatter_frames(allf, F, own.shape[1], dev)
    assert np.array_equal(got.numpy(), own)
    hdr = torch.from_numpy(_headers(own))
    gathered = cd.gather_headers(hdr)
    t = cd.max_over_ranks(float(rank + 1), dev)
    if rank == 0:
        np.save(result_path, np.concatenate([gathered.numpy().reshape(-1), [int(t)]]))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_batch_equals_single_rank(tmp_path):
    ws = 2
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(ws, _free_port(), out), nprocs=ws, join=True)
    res = np.load(out)
    gathered, tmax = res[:-1].reshape(ws * F, 8), int(res[-1])
    sys.path.insert(0, ROOT)
    import cones_perception_amd as cp
    single = _headers(cp.synth_frames(ws * F, first_frame=0, rings=RINGS, cols=COLS))
    assert np.array_equal(gathered, single)
    assert tmax == ws


def _bench(args, env=None):
    import json
    import subprocess
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=e)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` with no launcher environment starts two ranks itself (gloo in the
    dry run) and reports n_gpus 2 from rank 0, after a barrier and the max over ranks."""
    rc, line, err = _bench(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2 and line["dry_run"] is True
    assert line["config"]["parallelism"] == "frame-shard x2"
    # the rank census every real run carries: ranks all-gathered over the process group, the
    # backend, and the distinct devices behind them (none in a dry run)
    c = line["ranks"]
    assert c["ranks_seen"] == 2 and c["world_size_env"] == 2 and c["backend"] == "gloo"
    assert len(c["devices"]) == 2 and c["distinct_devices"] == 0


def test_bench_refuses_mismatched_world_size():
    rc, line, err = _bench(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0"})
    assert rc != 0 and line is None and "WORLD_SIZE=1" in err


def _merge_worker(rank, ws, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from cones_perception_amd import dist as cd
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    dev = torch.device("cpu")
    rng = np.random.default_rng(100 + rank)
    ok = True
    for it in range(20):
        # sector-minimum keys over the whole uint32 range (bit 31 set in about half), the
        # used-bin mask, and counts with bounds keys
        keys = rng.integers(0, 2 ** 32, 19, dtype=np.uint64).astype(np.uint32)
        keys[18] = rng.integers(0, 2 ** 18, dtype=np.uint64)
        counts = rng.integers(0, 2 ** 32, 9, dtype=np.uint64).astype(np.uint32)
        counts[:3] = rng.integers(0, 1 << 20, 3, dtype=np.uint64)
        host_k = cd.merge_tile_keys(keys, dev)
        dev_k = cd.merge_tile_keys_dev(torch.from_numpy(keys.view(np.int32).copy()), dev)
        ok &= np.array_equal(dev_k.numpy().view(np.uint32), host_k)
        host_c, sizes_h = cd.merge_tile_counts(counts, dev, per_rank=True)
        dev_c, sizes_d = cd.merge_tile_counts_dev(torch.from_numpy(counts.view(np.int32).copy()), dev)
        ok &= np.array_equal(dev_c, host_c) and sizes_h == sizes_d
    res = torch.tensor([int(ok)])
    dist.all_reduce(res, op=dist.ReduceOp.MIN)
    if rank == 0:
        np.save(result_path, res.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_device_side_tile_merges_equal_host_merges(tmp_path):
    """dist.merge_tile_keys_dev / merge_tile_counts_dev (the tiled C5 gather form's device-side
    merges, uint32 words carried as int32) against the host merges, world size 2 (gloo)."""
    out = str(tmp_path / "m.npy")
    mp.spawn(_merge_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert int(np.load(out)[0]) == 1
