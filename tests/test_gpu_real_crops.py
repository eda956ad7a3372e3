"""Real LiDAR points through the HIP path: the two labelled cone crops of the reference's
cones_clouds/cones.csv (tests/golden/cones_csv.npz, made by tests/golden/make_cones_csv.py; the
pickle with the other crops is not loaded) as detector input on their own, and placed into a
synthetic frame (as recorded, and copies moved along the track) for the fused pipeline, under
the reference's three parameter profiles. Every result bit-exact against the oracle."""
import os

import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import assert_same_detection

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cones_csv.npz")


def _crops():
    return np.load(FIXTURE)["points"].astype(np.float32)


def _frame_with_crops(frame, shifts):
    raw = cp.synth_frames(1, first_frame=frame, rings=64, cols=1024)
    pts = raw[0].view(np.float32).reshape(-1, 4).copy()
    crops = _crops()
    k = len(crops)
    for i, (dx, dy) in enumerate(shifts):   # every 4,099th slot: spread over the scan
        c = crops.copy()
        c[:, 0] += np.float32(dx)
        c[:, 1] += np.float32(dy)
        at = 100 + 4099 * i
        pts[at:at + k] = c
    return cp.PointCloud2.from_xyzi(pts)


@pytest.mark.parametrize("profile", ["simulation", "our", "fsai"])
def test_crops_alone_through_the_detector(profile):
    params = cp.load_params(profile)
    msg = cp.PointCloud2.from_xyzi(_crops())
    got = cp.ConeDetector(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_DETECT)
    assert_same_detection(got, ref, f"crops detect {profile}")


@pytest.mark.parametrize("profile", ["simulation", "our", "fsai"])
@pytest.mark.parametrize("frame", [0, 7])
def test_crops_in_a_frame_through_the_pipeline(profile, frame):
    params = cp.load_params(profile)
    shifts = [(0.0, 0.0), (1.0, 0.0), (2.5, -0.5), (4.0, 1.0), (-3.0, 0.5), (6.0, -2.0), (0.3, 2.0), (8.0, 0.0)]
    msg = _frame_with_crops(frame, shifts)
    got = cp.ConePipeline(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    assert_same_detection(got, ref, f"crops pipeline {profile} f{frame}")
    got_d = cp.ConeDetector(params).cloud_handler(msg)
    ref_d, _ = O.run(params, msg, O.MODE_DETECT)
    assert_same_detection(got_d, ref_d, f"crops detect-only {profile} f{frame}")
