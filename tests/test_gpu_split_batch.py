"""Batch frames as a front launch plus backend launches (cg_debug_route 6, cg_run_batch_split):
the streaming front (pass 1, thresholds, pass 2, survivors to the frame's HBM slot), the
256-lane backend launch (cg_back.hip) and the 512-lane one for the frames it hands on.
Every frame bit-exact against the oracle in PCL's voxel order, and identical to the default
fused one-workgroup-per-frame kernel, across the backend launches' branches:
LDS (M <= 392) with all-pairs (V <= 128) or neighbour-grid clustering, the HBM slot (M > 392),
zero pads, C1-sized frames (32 points per lane), the detector-only mode and the known-answer
clouds as one-frame batches."""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import assert_same_detection
from kat_clouds import all_kats

pytestmark = pytest.mark.gpu


def _run(params, raw, n_points, mode=cp.CG_MODE_PIPELINE, route=0):
    import torch
    d = torch.from_numpy(np.ascontiguousarray(raw)).cuda()
    eng = cp.BatchEngine(params)
    if route:
        eng.debug_route(route)
    eng.run(d.data_ptr(), raw.shape[0], n_points, 16, mode=mode, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return [eng.fetch(f) for f in range(raw.shape[0])]


def _mixed(rings=64):
    return np.stack([cp.synth_frames(1, first_frame=f, rings=rings, cols=1024, clutter=c, cones_per_row=k)[0]
                     for f, c, k in ((0, 0, 5), (1, 0, 8), (2, 20, 8), (3, 60, 10), (4, 200, 10), (5, 0, 5),
                                     (6, 40, 12), (7, 0, 3))])


@pytest.mark.parametrize("over", [{}, {"distance_treshold_min": 0.0}], ids=["default", "zero-pads"])
@pytest.mark.parametrize("rings", [64, 16])
def test_split_batch_matches_oracle_and_fused(over, rings):
    params = cp.load_params("simulation", over)
    raw = _mixed(rings)
    n = rings * 1024
    split = _run(params, raw, n, route=6)
    fused = _run(params, raw, n)
    ms, vs = [], []
    for f in range(raw.shape[0]):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE, O.ORDER_PCL)
        assert_same_detection(split[f], ref, f"split batch frame {f}")
        assert_same_detection(fused[f], ref, f"fused batch frame {f}")
        ms.append(ref.n_filtered)
        vs.append(ref.voxels.shape[0])
    if rings == 64 and not over:   # the backend launch's branches were all taken
        assert min(ms) <= 392 < max(ms), ms
        assert any(v > 128 and m <= 392 for v, m in zip(vs, ms)) or max(vs) > 128, (ms, vs)


def test_split_batch_detector_mode():
    params = cp.load_params("simulation")
    raw = _mixed()
    got = _run(params, raw, 65536, mode=cp.CG_MODE_DETECT, route=6)
    for f in range(raw.shape[0]):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_DETECT, O.ORDER_PCL)
        assert_same_detection(got[f], ref, f"detect batch frame {f}")


def test_split_batch_point_order():
    params = cp.load_params("simulation")
    raw = _mixed()
    import torch
    d = torch.from_numpy(raw).cuda()
    eng = cp.BatchEngine(params).set_voxel_order(cp.CG_VOXEL_ORDER_POINT).debug_route(6)
    eng.run(d.data_ptr(), raw.shape[0], 65536, 16)
    torch.cuda.synchronize()
    for f in range(raw.shape[0]):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE, O.ORDER_STABLE)
        assert_same_detection(eng.fetch(f), ref, f"point-order batch frame {f}")


@pytest.mark.parametrize("kat", all_kats(), ids=lambda k: k[0])
def test_kats_as_one_frame_batches(kat):
    name, pts, over, _ = kat
    params = cp.load_params("simulation", over)
    msg = cp.PointCloud2.from_xyzi(pts)
    raw = np.frombuffer(msg.data, np.uint8).reshape(1, -1)
    n = raw.shape[1] // 16
    if n == 0 or n > 65536:
        pytest.skip("batch frames hold 1-65,536 points")
    got = _run(params, raw, n, route=6)[0]
    ref, _ = O.run(params, msg, O.MODE_PIPELINE, O.ORDER_PCL)
    assert_same_detection(got, ref, f"{name} as a batch")


def test_split_streams_rotation_matches_oracle():
    """cg_run_batch_split: fronts on two streams, backends on a third, four handles in
    rotation over eight batches (each handle's next front waits for its backends); every
    frame of the last round bit-exact."""
    import torch
    params = cp.load_params("simulation")
    raw = _mixed()
    d = [torch.from_numpy(np.roll(raw, k, axis=0).copy()).cuda() for k in range(4)]
    engines = [cp.BatchEngine(params) for _ in range(4)]
    fronts = [torch.cuda.Stream() for _ in range(2)]
    back = torch.cuda.Stream()
    for i in range(8):
        engines[i % 4].run(d[i % 4].data_ptr(), raw.shape[0], 65536, 16, stream=fronts[i % 2].cuda_stream,
                           back_stream=back.cuda_stream)
    torch.cuda.synchronize()
    refs = [O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE, O.ORDER_PCL)[0] for f in range(raw.shape[0])]
    for k in range(4):
        for f in range(raw.shape[0]):
            assert_same_detection(engines[k].fetch(f), refs[(f - k) % raw.shape[0]], f"handle {k} frame {f}")
