"""Colour classifier on the GPU (cg_classify_colors) against the CPU restatement
(tests/colornet_ref.py): to_image bit-exact, probabilities within 2e-5 of the float64
network (the reference's own TFLite outputs are unpinned: TensorFlow is not available), the
service's colours and response rules identical. Clouds: real re-crops of synthetic frames
plus edge cases (empty, one point, duplicate pixels, >256 points, rows out of the image,
intensities out of range)."""
import os

import numpy as np
import pytest

import colornet_ref as R
import cones_perception_amd as cp
from cones_perception_amd import colornet

pytestmark = pytest.mark.gpu
W = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dam_net_weights.npy"))
PROB_TOL = 2e-5


def _cone(n, seed, x0=6.0, y0=1.0):
    g = np.random.default_rng(seed)
    pts = np.zeros((n, 4), np.float32)
    pts[:, 0] = x0 + g.uniform(-0.12, 0.12, n)
    pts[:, 1] = y0 + g.uniform(-0.12, 0.12, n)
    pts[:, 2] = g.uniform(-0.5, -0.15, n)
    pts[:, 3] = g.uniform(0, 255, n)
    return pts


def _compare(clouds):
    clf = colornet.ColorClassifier(W)
    col, pr, img = clf.classify(clouds, want_images=True)
    ref = R.classify(clouds, W)
    for k, (rc, rp, ri) in enumerate(ref):
        assert col[k] == rc or (rp is not None and abs(rp.max() - 0.8) < 1e-4), (k, col[k], rc)
        if ri is not None:
            assert np.array_equal(img[k], ri), f"cloud {k}: image differs"
            assert np.max(np.abs(pr[k] - rp)) < PROB_TOL, (k, pr[k], rp)
    return col, pr


def test_recrops_of_synthetic_frames():
    params = cp.load_params("simulation")
    pipe = cp.ConePipeline(params, device=0)
    clouds = []
    for f in range(4):
        raw = cp.synth_frames(1, first_frame=f, rings=64, cols=1024, cones_per_row=6)
        det = pipe.cloud_handler(cp.frame_cloud(raw[0]))
        clouds += [c for c in pipe.recrop(det.centroids)]
    assert len(clouds) >= 8 and sum(len(c) for c in clouds) > 100
    col, pr = _compare(clouds)
    assert (col >= 0).all()


def test_edge_clouds():
    base = _cone(50, 3)
    dup = np.vstack([base, base[::7]]).astype(np.float32)          # later points overwrite pixels
    big = _cone(1500, 4, 8.0, -2.0)                                # more points than lanes
    far = base.copy()
    far[5, 2] = 40.0                                               # row outside the image
    hot = base.copy()
    hot[9, 3] = 300.0                                              # interp1d range error
    edge = base.copy()
    edge[:, 3] = np.float32(255.0)                                 # the range's end is allowed
    clouds = [base, np.zeros((0, 4), np.float32), base[:1], dup, big, far, hot, edge, _cone(7, 5, -3.0, 4.0)]
    col, _ = _compare(clouds)
    assert col[1] == colornet.SKIPPED and col[5] == colornet.INDEX_ERROR and col[6] == colornet.RANGE_ERROR


def test_service_response_rules():
    clf = colornet.ColorClassifier(W)
    clouds = [_cone(30, s) for s in range(6)]
    clouds.insert(2, np.zeros((0, 4), np.float32))
    got = clf.handle_classify_color([cp.to_ros_msg(c) for c in clouds])
    want = [c for c, _, _ in R.classify(clouds, W) if c != colornet.SKIPPED]
    assert got == want and len(got) == 6
    bad = _cone(30, 9)
    bad[4, 2] = 40.0
    with pytest.raises(IndexError):
        clf.handle_classify_color([clouds[0], bad])


def test_detector_node_with_gpu_classifier():
    """The whole detector callback with the service served in process: every cone that needs a
    colour gets the classifier's answer (tracking then publishes it)."""
    params = cp.load_params("simulation")
    clf = colornet.ColorClassifier(W)
    node = cp.ConeDetectorNode(params, classifier=clf.handle_classify_color, fused_ground_removal=True)
    for f in range(3):
        raw = cp.synth_frames(1, first_frame=f, rings=64, cols=1024, cones_per_row=6)
        out = node.cloud_handler(cp.frame_cloud(raw[0]))
        assert len(out) == 4
    assert sum(m.width for m in out) > 0


def test_reference_csv_crops():
    """The labelled crops of the reference's cones_clouds/cones.csv through cg_classify_colors:
    images bit-exact, probabilities within PROB_TOL of the float64 restatement."""
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cones_csv.npz"))
    o = z["offsets"]
    clouds = [z["points"][o[i]:o[i + 1]] for i in range(len(o) - 1)]
    col, _ = _compare(clouds)
    assert list(col) == [1, 1]   # human labels [1, 2]: see test_colornet.test_reference_csv_crops_through_the_restatement
