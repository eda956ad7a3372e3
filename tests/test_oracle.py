"""The CPU restatement (oracle/) against the independent numpy restatement, on synthetic
C1-sized frames and on the PCL-order (std::sort) vs stable-order voxel summation."""
import numpy as np
import pytest

import cones_perception_amd as cp
import np_reference as R
import oracle_py as O

PRM = {**cp.GROUND_PARAMS, **cp.PROFILES["simulation"]}


def _compare(det, ref, ctx):
    assert det.n_kept == ref["K"], ctx
    assert det.n_filtered == ref["M"], ctx
    assert np.array_equal(det.voxels.view(np.uint32), ref["vox"].view(np.uint32)), ctx
    assert [list(c) for c in det.clusters] == ref["clusters"], ctx
    assert np.array_equal(det.centroids.view(np.uint32), ref["centroids"].view(np.uint32)), ctx


@pytest.mark.parametrize("frame", range(3))
def test_oracle_matches_numpy_c1(frame):
    raw = cp.synth_frames(1, first_frame=frame, rings=16, cols=1024)
    msg = cp.frame_cloud(raw[0])
    params = cp.load_params("simulation")
    det, _ = O.run(params, msg, O.MODE_PIPELINE, O.ORDER_STABLE)
    ref = R.pipeline(msg.xyzi(), PRM, ground=True)
    assert len(ref["clusters"]) > 0
    _compare(det, ref, f"frame {frame}")


def test_oracle_matches_numpy_detector_only():
    raw = cp.synth_frames(1, first_frame=4, rings=16, cols=1024)
    msg = cp.frame_cloud(raw[0])
    params = cp.load_params("simulation")
    det, _ = O.run(params, msg, O.MODE_DETECT, O.ORDER_STABLE)
    _compare(det, R.pipeline(msg.xyzi(), PRM, ground=False), "detect")


def test_oracle_matches_numpy_our_profile():
    raw = cp.synth_frames(1, first_frame=6, rings=16, cols=1024)
    msg = cp.frame_cloud(raw[0])
    prm = {**cp.GROUND_PARAMS, **cp.PROFILES["our"]}
    det, _ = O.run(cp.load_params("our"), msg, O.MODE_PIPELINE, O.ORDER_STABLE)
    _compare(det, R.pipeline(msg.xyzi(), prm, ground=True), "our")


def test_ground_output_layout():
    raw = cp.synth_frames(1, first_frame=1, rings=16, cols=1024)
    msg = cp.frame_cloud(raw[0])
    g, hdr = O.run(cp.load_params("simulation"), msg, O.MODE_GROUND)
    pts = g.view(np.float32).reshape(-1, 8)
    ref, K = R.ground_remove(msg.xyzi(), -0.1)
    assert int(hdr[1]) == K
    assert np.array_equal(pts[:, [0, 1, 2, 4]].view(np.uint32), ref.view(np.uint32))
    assert np.all(pts[:, 3] == 1.0)          # PointXYZI data[3]
    assert not pts[K:, [0, 1, 2, 4]].any()   # PointXYZI() padding


def test_pcl_sort_order_vs_stable_order_c2():
    """PCL's unstable std::sort sums voxels in introsort order; the device sums in point order.
    Count frames where that changes anything (cluster sets or centroid bits)."""
    params = cp.load_params("simulation")
    raw = cp.synth_frames(6, first_frame=0, rings=64, cols=1024)
    diff_sets = diff_bits = 0
    for f in range(raw.shape[0]):
        msg = cp.frame_cloud(raw[f])
        a, _ = O.run(params, msg, O.MODE_PIPELINE, O.ORDER_STABLE)
        b, _ = O.run(params, msg, O.MODE_PIPELINE, O.ORDER_PCL)
        diff_sets += not np.array_equal(a.cluster_indices, b.cluster_indices)
        diff_bits += not np.array_equal(a.voxels.view(np.uint32), b.voxels.view(np.uint32))
    assert diff_sets == 0
    print(f"voxel-bit differences stable vs PCL order: {diff_bits} / {raw.shape[0]} frames")
