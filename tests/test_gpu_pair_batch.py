"""Pipeline batches as two half-frame workgroups per frame (cg_debug_route 7, cg_pair.hip):
both halves stream pass 1, the first to finish publishes its sector keys, codes and filter bits
into the frame's scratch slot, the second merges them and runs the frame's tail. Every frame
bit-exact against the oracle in PCL's voxel order (and in point order), across the branches:
the pair kernel's LDS backend (M <= 512) with all-pairs (V <= 128) or neighbour-grid
clustering, the listed frames of the launches after it (512 < M <= 1,024: cg_back_big; more:
cg_back_list on the HBM slot), zero pads, partial second halves, generic point layouts and
repeated batches on one handle (the exchange words' epochs)."""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import assert_same_detection

pytestmark = pytest.mark.gpu

# (first_frame, clutter, cones_per_row): detector points 243, 244, 1525, 4058, 290, 643, 364, 444
FRAMES = ((0, 0, 5), (1, 0, 8), (2, 20, 8), (3, 60, 10), (8, 5, 8), (9, 10, 8), (10, 2, 10), (11, 4, 12))


def _frames(n_points=65536):
    raw = np.stack([cp.synth_frames(1, first_frame=f, rings=64, cols=1024, clutter=c, cones_per_row=k)[0]
                    for f, c, k in FRAMES])
    return np.ascontiguousarray(raw[:, :n_points * 16])


def _run(eng, raw, n_points, step=16, offsets=(0, 4, 8, 12)):
    import torch
    d = torch.from_numpy(np.ascontiguousarray(raw)).cuda()
    eng.run(d.data_ptr(), raw.shape[0], n_points, step, stream=torch.cuda.current_stream().cuda_stream,
            offsets=offsets)
    torch.cuda.synchronize()
    return [eng.fetch(f) for f in range(raw.shape[0])]


def _check(params, raw, got, order=O.ORDER_PCL, what="pair"):
    ms, vs = [], []
    for f in range(raw.shape[0]):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE, order)
        assert_same_detection(got[f], ref, f"{what} frame {f}")
        assert not got[f].flags & cp.CG_F_PAIR_TIMEOUT, f"{what} frame {f}: the second half timed out"
        ms.append(ref.n_filtered)
        vs.append(ref.voxels.shape[0])
    return ms, vs


@pytest.mark.parametrize("over", [{}, {"distance_treshold_min": 0.0}], ids=["default", "zero-pads"])
@pytest.mark.parametrize("n_points", [65536, 40000])
def test_pair_batch_matches_oracle(over, n_points):
    params = cp.load_params("simulation", over)
    raw = _frames(n_points)
    got = _run(cp.BatchEngine(params).debug_route(7), raw, n_points)
    ms, vs = _check(params, raw, got)
    if n_points == 65536 and not over:   # every branch taken
        assert any(m <= 512 and v > 128 for m, v in zip(ms, vs)), (ms, vs)
        assert any(m <= 512 and v <= 128 for m, v in zip(ms, vs)), (ms, vs)
        assert any(512 < m <= 1024 for m in ms) and any(m > 1024 for m in ms), ms


def test_pair_batch_point_order():
    params = cp.load_params("simulation")
    raw = _frames()
    eng = cp.BatchEngine(params).set_voxel_order(cp.CG_VOXEL_ORDER_POINT).debug_route(7)
    _check(params, raw, _run(eng, raw, 65536), O.ORDER_STABLE, "point-order pair")


def test_pair_batch_generic_layout():
    """20-byte points (x, y, z, pad, intensity): the generic-layout instantiation."""
    params = cp.load_params("simulation")
    raw = _frames()
    pts = raw.view(np.float32).reshape(raw.shape[0], -1, 4)
    wide = np.zeros((raw.shape[0], pts.shape[1], 5), np.float32)
    wide[..., :3] = pts[..., :3]
    wide[..., 4] = pts[..., 3]
    w8 = wide.view(np.uint8).reshape(raw.shape[0], -1)
    got = _run(cp.BatchEngine(params).debug_route(7), w8, 65536, 20, (0, 4, 8, 16))
    _check(params, raw, got, what="generic-layout pair")


def test_pair_batches_repeat_on_one_handle():
    """Eight batches on one handle, the frames rotated each time: the exchange words' tickets
    reset and the ready words' epochs advance; every batch bit-exact, and equal to the fused
    kernel's results."""
    params = cp.load_params("simulation")
    raw = _frames()
    refs = [O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE, O.ORDER_PCL)[0] for f in range(raw.shape[0])]
    eng = cp.BatchEngine(params).debug_route(7)
    fused = cp.BatchEngine(params)
    for k in range(8):
        rolled = np.roll(raw, k, axis=0)
        got = _run(eng, rolled, 65536)
        for f in range(raw.shape[0]):
            assert_same_detection(got[f], refs[(f - k) % raw.shape[0]], f"batch {k} frame {f}")
    got_f = _run(fused, rolled, 65536)
    for f in range(raw.shape[0]):
        assert_same_detection(got[f], got_f[f], f"pair vs fused frame {f}")


def test_pair_single_frame_batches():
    """One-frame batches (grid of 16 workgroups, 14 of them idle) and an odd frame count."""
    params = cp.load_params("simulation")
    raw = _frames()
    eng = cp.BatchEngine(params).debug_route(7)
    for f in (0, 5):
        got = _run(eng, raw[f:f + 1], 65536)[0]
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE, O.ORDER_PCL)
        assert_same_detection(got, ref, f"single frame {f}")
    got = _run(eng, raw[:5], 65536)
    _check(params, raw[:5], got, what="five-frame pair")
