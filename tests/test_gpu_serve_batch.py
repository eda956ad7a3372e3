"""Served batches (cg_debug_route 8): the front launch publishes each frame's survivors through
device-coherent stores and a publish word; the backend launch (cg_serve_kernel) runs beside it,
each workgroup taking its frame as soon as it is published. Every frame bit-exact against the
oracle in PCL's voxel order and in point order, across the backend's branches (LDS up to 392
detector points with all-pairs or neighbour-grid clustering; the listed frames of the launches
after it: up to 1,024 in cg_back_big, more on the HBM slot), with the backends on the front's
stream and on a stream of their own, and over repeated batches on rotating handles (the publish
words' epochs)."""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import assert_same_detection

pytestmark = pytest.mark.gpu

# (first_frame, clutter, cones_per_row): detector points 243, 244, 1525, 4058, 290, 643, 364, 444
FRAMES = ((0, 0, 5), (1, 0, 8), (2, 20, 8), (3, 60, 10), (8, 5, 8), (9, 10, 8), (10, 2, 10), (11, 4, 12))


def _frames(rings=64):
    return np.stack([cp.synth_frames(1, first_frame=f, rings=rings, cols=1024, clutter=c, cones_per_row=k)[0]
                     for f, c, k in FRAMES])


def _check(params, raw, got, order=O.ORDER_PCL, what="served"):
    ms, vs = [], []
    for f in range(raw.shape[0]):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE, order)
        assert_same_detection(got[f], ref, f"{what} frame {f}")
        ms.append(ref.n_filtered)
        vs.append(ref.voxels.shape[0])
    return ms, vs


@pytest.mark.parametrize("back", [False, True], ids=["one-stream", "back-stream"])
@pytest.mark.parametrize("over", [{}, {"distance_treshold_min": 0.0}], ids=["default", "zero-pads"])
@pytest.mark.parametrize("rings", [64, 16])
def test_served_batch_matches_oracle(back, over, rings):
    import torch
    params = cp.load_params("simulation", over)
    raw = _frames(rings)
    n = rings * 1024
    d = torch.from_numpy(raw).cuda()
    eng = cp.BatchEngine(params).debug_route(8)
    front = torch.cuda.Stream()
    bs = torch.cuda.Stream() if back else None
    eng.run(d.data_ptr(), raw.shape[0], n, 16, stream=front.cuda_stream, back_stream=bs.cuda_stream if back else 0)
    torch.cuda.synchronize()
    ms, vs = _check(params, raw, [eng.fetch(f) for f in range(raw.shape[0])])
    if rings == 64 and not over:   # every branch taken
        assert any(m <= 392 and v > 128 for m, v in zip(ms, vs)), (ms, vs)
        assert any(m <= 392 and v <= 128 for m, v in zip(ms, vs)), (ms, vs)
        assert any(392 < m <= 1024 for m in ms) and any(m > 1024 for m in ms), ms


def test_served_batch_point_order_and_detect():
    import torch
    params = cp.load_params("simulation")
    raw = _frames()
    d = torch.from_numpy(raw).cuda()
    eng = cp.BatchEngine(params).set_voxel_order(cp.CG_VOXEL_ORDER_POINT).debug_route(8)
    front, back = torch.cuda.Stream(), torch.cuda.Stream()
    eng.run(d.data_ptr(), raw.shape[0], 65536, 16, stream=front.cuda_stream, back_stream=back.cuda_stream)
    torch.cuda.synchronize()
    _check(params, raw, [eng.fetch(f) for f in range(raw.shape[0])], O.ORDER_STABLE, "point-order served")
    eng2 = cp.BatchEngine(params).debug_route(8)
    eng2.run(d.data_ptr(), raw.shape[0], 65536, 16, mode=cp.CG_MODE_DETECT, stream=front.cuda_stream,
             back_stream=back.cuda_stream)
    torch.cuda.synchronize()
    for f in range(raw.shape[0]):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_DETECT, O.ORDER_PCL)
        assert_same_detection(eng2.fetch(f), ref, f"detect served frame {f}")


def test_served_batches_rotation():
    """Fronts on three streams, backends on one, four handles in rotation over twelve batches
    (each handle's next front waits for its backends; the publish words carry each batch's
    epoch). Every frame of every handle's last batch bit-exact, and a large batch of 256 C3
    frames against the fused kernel."""
    import torch
    params = cp.load_params("simulation")
    raw = _frames()
    d = [torch.from_numpy(np.roll(raw, k, axis=0).copy()).cuda() for k in range(4)]
    engines = [cp.BatchEngine(params).debug_route(8) for _ in range(4)]
    fronts = [torch.cuda.Stream() for _ in range(3)]
    back = torch.cuda.Stream()
    for i in range(12):
        engines[i % 4].run(d[i % 4].data_ptr(), raw.shape[0], 65536, 16, stream=fronts[i % 3].cuda_stream,
                           back_stream=back.cuda_stream)
    torch.cuda.synchronize()
    refs = [O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE, O.ORDER_PCL)[0] for f in range(raw.shape[0])]
    for k in range(4):
        for f in range(raw.shape[0]):
            assert_same_detection(engines[k].fetch(f), refs[(f - k) % raw.shape[0]], f"handle {k} frame {f}")
    big = cp.synth_frames(256, first_frame=7)
    db = torch.from_numpy(big).cuda()
    served, fused = cp.BatchEngine(params).debug_route(8), cp.BatchEngine(params)
    for _ in range(2):
        served.run(db.data_ptr(), 256, 65536, 16, stream=fronts[0].cuda_stream, back_stream=back.cuda_stream)
    fused.run(db.data_ptr(), 256, 65536, 16, stream=fronts[1].cuda_stream)
    torch.cuda.synchronize()
    for f in range(256):
        assert_same_detection(served.fetch(f), fused.fetch(f), f"256-frame batch frame {f}")
