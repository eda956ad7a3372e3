"""The batch engine's host side on the GPU: cg_run_batches (many batch calls in one crossing of
the ABI, as bench.py's timed region enqueues them), a handle's calls ordered across streams,
the single-frame staging retry, and the tile backend under the diagnostic route that forces the
global backend with one partition level (route 5). Every result is checked bit for bit against
the CPU restatement in PCL's voxel order."""
import time

import pytest

import cones_perception_amd as cp
from cones_perception_amd import _abi
import oracle_py as O
from helpers import assert_same_detection

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def params():
    return cp.load_params("simulation")


def _refs(params, raw):
    return [O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE)[0] for f in range(raw.shape[0])]


def test_run_batches_rotation_matches_oracle(params):
    """Nine calls over three handles and three streams in one cg_run_batches call (bench.py's
    rotation): each handle's last batch, every frame, against the oracle."""
    import torch
    nf = 12
    raws = [cp.synth_frames(nf, first_frame=300 + 40 * k, rings=64, cols=1024, clutter=10 * k, cones_per_row=6)
            for k in range(3)]
    ds = [torch.from_numpy(r).cuda() for r in raws]
    engines = [cp.BatchEngine(params) for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    n = 9
    q = cp.BatchQueue([engines[i % 3] for i in range(n)],
                      [cp.batch_desc(ds[i % 3].data_ptr(), nf, 65536, 16) for i in range(n)],
                      [streams[i % 3].cuda_stream for i in range(n)])
    assert q.run() == n
    torch.cuda.synchronize()
    for k in range(3):
        refs = _refs(params, raws[k])
        for f in range(nf):
            assert_same_detection(engines[k].fetch(f), refs[f], f"queue handle {k} frame {f}")


def test_run_batches_checks_every_call_first(params):
    """A bad call anywhere refuses the whole sequence: nothing is enqueued (n_done = 0)."""
    import torch
    raw = cp.synth_frames(2, first_frame=5, rings=64, cols=1024)
    d = torch.from_numpy(raw).cuda()
    eng = cp.BatchEngine(params)
    good = cp.batch_desc(d.data_ptr(), 2, 65536, 16)
    bad = cp.batch_desc(d.data_ptr(), 2, 65536, 6)   # point_step not a multiple of 4
    q = cp.BatchQueue([eng, eng], [good, bad], [0, 0])
    with pytest.raises(_abi.CgError):
        q.run()
    assert q._done.value == 0
    eng.run(d.data_ptr(), 2, 65536, 16)   # the handle stays usable
    ref = _refs(params, raw)
    for f in range(2):
        assert_same_detection(eng.fetch(f), ref[f], f"after refusal frame {f}")


def test_handle_calls_ordered_across_streams(params):
    """A handle's second batch on another stream waits for its first (same slots): dense
    frames on stream A, then light frames on stream B; the second batch's results against the
    oracle."""
    import torch
    heavy = cp.synth_frames(64, first_frame=7, rings=64, cols=1024, clutter=200, cones_per_row=10)
    light = cp.synth_frames(8, first_frame=70, rings=64, cols=1024)
    dh, dl = torch.from_numpy(heavy).cuda(), torch.from_numpy(light).cuda()
    eng = cp.BatchEngine(params)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    eng.run(dh.data_ptr(), 64, 65536, 16, stream=sa.cuda_stream)
    eng.run(dl.data_ptr(), 8, 65536, 16, stream=sb.cuda_stream)
    ref = _refs(params, light)
    for f in range(8):
        assert_same_detection(eng.fetch(f), ref[f], f"second stream frame {f}")


def test_staging_timeout_reruns_by_dma(params):
    """Route 6 withholds every chunk's publish word, so each chunk workgroup gives up after
    200 ms and the call re-runs the frame with its input by DMA: the result is exact (the
    call is slower, never failed)."""
    pipe = cp.ConePipeline(params)
    raw = cp.synth_frames(1, first_frame=21, rings=64, cols=1024)
    msg = cp.frame_cloud(raw[0])
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    pipe.debug_route(6)
    t0 = time.perf_counter()
    got = pipe.cloud_handler(msg)
    dt = time.perf_counter() - t0
    assert dt >= 0.19, f"{dt:.3f} s: the chunk workgroups did not wait for their publish words"
    assert_same_detection(got, ref, "after the staging timeout")
    pipe.debug_route(0)
    assert_same_detection(pipe.cloud_handler(msg), ref, "zero-copy again")


def test_split_give_up_reruns_in_one_workgroup(params):
    """Route 9: chunk workgroup 0 of the split launch gives up waiting for the other chunks at
    once (as after CG_SPLIT_TIMEOUT), so the frame's counts are void (header word 7) and the
    call re-runs it in one workgroup: the result is exact (a void frame would have no
    survivors), and the state words the last chunk reset leave the next split call clean."""
    pipe = cp.ConePipeline(params)
    for frame in (22, 23):
        raw = cp.synth_frames(1, first_frame=frame, rings=64, cols=1024)
        msg = cp.frame_cloud(raw[0])
        ref, _ = O.run(params, msg, O.MODE_PIPELINE)
        assert ref.n_filtered > 0 and len(ref.centroids) > 0
        pipe.debug_route(9)
        assert_same_detection(pipe.cloud_handler(msg), ref, f"frame {frame} after the give-up")
        pipe.debug_route(0)
        assert_same_detection(pipe.cloud_handler(msg), ref, f"frame {frame} split again")


def test_tile_backend_keeps_route5(params):
    """cg_tile_backend_own under route 5 (global backend, PCL sort cut after one partition
    level): the route reaches the tile protocol, and the result is exact."""
    import torch
    from cones_perception_amd import dist as cd
    raw = cp.synth_frames(1, first_frame=9, rings=128, cols=2048, clutter=60, cones_per_row=12)
    n = raw.shape[1] // 16
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(raw[0].copy()).to(dev)
    eng = cp.BatchEngine(params, device=0)
    eng.debug_route(5)
    got = cd.run_tiled_frame(eng, d.data_ptr(), 0, n, n, dev, halo=False)
    ref, hdr = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE, O.ORDER_PCL)
    assert int(hdr[2]) > 4096   # M past the LDS leaf: the cut leaves leaves for the HBM fallback
    assert_same_detection(got, ref, "tile backend route 5")
    assert got.flags & cp.CG_F_GLOBAL_SCRATCH
