"""Chunked batches (cg_debug_route 7): every frame of a batch split over one workgroup per
4,096-point chunk in one launch of the split kernel; each frame's last chunk runs its backend.
Frames are dealt to XCDs in groups of eight, so batches whose frame count is not a multiple of
eight leave padding workgroups. Every frame is checked bit for bit against the CPU restatement
in PCL's voxel order (src/ground_removal.cpp:50-89, src/cone_detection.cpp:130-280)."""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import assert_same_detection

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def params():
    return cp.load_params("simulation")


def _run(params, raw, mode=cp.CG_MODE_PIPELINE, point_step=16, n_points=65536, repeat=1, offsets=(0, 4, 8, 12)):
    import torch
    d = torch.from_numpy(raw).cuda()
    eng = cp.BatchEngine(params)
    eng.debug_route(7)
    for _ in range(repeat):   # the per-frame state words reset themselves between launches
        eng.run(d.data_ptr(), raw.shape[0], n_points, point_step, mode=mode, offsets=offsets,
                stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return eng


@pytest.mark.parametrize("nf", [1, 13, 64])
def test_chunk_batch_matches_oracle(params, nf):
    raw = cp.synth_frames(nf, first_frame=500, rings=64, cols=1024, cones_per_row=6)
    eng = _run(params, raw, repeat=2)
    for f in range(nf):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE)
        got = eng.fetch(f)
        assert_same_detection(got, ref, f"chunked frame {f}/{nf}")
        assert eng.results().n_frames == nf


def test_chunk_batch_mixed_backends(params):
    """LDS-path and HBM-scratch-path frames (M > 1,024) in one chunked batch."""
    raws = [cp.synth_frames(1, first_frame=f, rings=64, cols=1024, clutter=c, cones_per_row=8)[0]
            for f, c in ((0, 0), (1, 60), (2, 20), (3, 200), (4, 0), (5, 200), (6, 0), (7, 60), (8, 0))]
    raw = np.stack(raws)
    eng = _run(params, raw)
    for f in range(raw.shape[0]):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE)
        assert_same_detection(eng.fetch(f), ref, f"chunked mixed frame {f}")


def test_chunk_batch_detect_mode_and_pcl32(params):
    """The detector's input mode, and the 32-byte PointXYZI layout (generic loads)."""
    raw = cp.synth_frames(10, first_frame=40, rings=64, cols=1024, cones_per_row=7)
    eng = _run(params, raw, mode=cp.CG_MODE_DETECT)
    for f in range(10):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_DETECT)
        assert_same_detection(eng.fetch(f), ref, f"chunked detect frame {f}")
    raw32 = cp.synth_frames(9, first_frame=60, rings=64, cols=1024, point_step=32)
    eng = _run(params, raw32, point_step=32, offsets=(0, 4, 8, 16))   # PointXYZI: intensity at 16
    for f in range(9):
        ref, _ = O.run(params, cp.frame_cloud(raw32[f], 32), O.MODE_PIPELINE)
        assert_same_detection(eng.fetch(f), ref, f"chunked pcl32 frame {f}")


def test_chunk_batch_ragged_frames(params):
    """Frames of 40,000 points (the last chunk partial) and of 1,000 points (one chunk)."""
    for rings, cols in ((40, 1000), (1, 1000)):
        raw = cp.synth_frames(11, first_frame=80, rings=rings, cols=cols)
        eng = _run(params, raw, n_points=rings * cols)
        for f in range(11):
            ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE)
            assert_same_detection(eng.fetch(f), ref, f"chunked {rings}x{cols} frame {f}")
