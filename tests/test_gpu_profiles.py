"""GPU parity under the reference's other two parameter profiles
(config/cones_detection_params_our.yaml: angle threshold 90 deg, i.e. a filter edge at exactly
+-pi/2, level -0.5, clusters [3, 50]; config/cones_detection_params_fsai.yaml: level -0.09),
through the pipeline, the detector and the ground node, on synthetic C2 frames, a cluttered
frame, the large path, and the adversarial edge frames (tests/edge_frames.py) with their
angle-filter probes at +-90 deg. Bit for bit against the oracle (PCL voxel order)."""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from edge_frames import BANDS, sector_edge_frame
from helpers import assert_same_detection

pytestmark = pytest.mark.gpu

PROFILES = ["our", "fsai"]


def _all_modes(params, msg, ctx):
    out = cp.GroundRemover(params).cloud_handler(msg)
    ref, hdr = O.run(params, msg, O.MODE_GROUND)
    assert out.n_kept == int(hdr[1]), ctx
    g = out.data.view(np.float32).reshape(-1, 8)
    r = ref.view(np.float32).reshape(-1, 8)
    assert np.array_equal(g[:, :5].view(np.uint32), r[:, :5].view(np.uint32)), ctx
    dets = {}
    for mode, eng, om in (("pipeline", cp.ConePipeline, O.MODE_PIPELINE), ("detect", cp.ConeDetector, O.MODE_DETECT)):
        got = eng(params).cloud_handler(msg)
        want, _ = O.run(params, msg, om)
        assert_same_detection(got, want, f"{ctx} {mode}")
        dets[mode] = got
    return dets


@pytest.mark.parametrize("profile", PROFILES)
@pytest.mark.parametrize("rings,cols,clutter,frame", [(64, 1024, 0, 0), (64, 1024, 0, 7), (64, 1024, 60, 3),
                                                      (128, 1024, 20, 1)])
def test_profile_frames_match_oracle(profile, rings, cols, clutter, frame):
    params = cp.load_params(profile)
    raw = cp.synth_frames(1, first_frame=frame, rings=rings, cols=cols, clutter=clutter, cones_per_row=8)
    _all_modes(params, cp.frame_cloud(raw[0]), f"{profile} {rings}x{cols} clutter {clutter} f{frame}")


@pytest.mark.parametrize("order", ["angle", "shuffled"])
@pytest.mark.parametrize("band", range(len(BANDS)))
def test_our_profile_edge_frames_at_90_degrees(band, order):
    """`our`: the angle filter removes atan2f(y, x) <= -pi/2 or >= pi/2 (double compares of the
    float angle against +-90 deg in radians); probes within 1e-8..1e-2 rad of both edges."""
    params = cp.load_params("our")
    pts = sector_edge_frame(band, order, 65536, seed=3, theta_deg=90.0)
    # lift the probes into `our`'s band: level -0.5, 0.7 <= distance <= 7
    msg = cp.PointCloud2.from_xyzi(pts)
    dets = _all_modes(params, msg, f"our 90deg band {BANDS[band]} {order}")
    assert dets["detect"].n_filtered > 0


def test_our_profile_edge_frame_large_path():
    params = cp.load_params("our")
    pts = sector_edge_frame(2, "angle", 131072, seed=5, theta_deg=90.0)
    _all_modes(params, cp.PointCloud2.from_xyzi(pts), "our 90deg large")
