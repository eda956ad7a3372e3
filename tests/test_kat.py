"""Known-answer clouds (tests/kat_clouds.py) on the CPU restatement, cross-checked against the
independent numpy restatement, with hand-derived expectations for each edge semantic."""
import numpy as np
import pytest

import cones_perception_amd as cp
import kat_clouds as KC
import np_reference as R
import oracle_py as O

KATS = KC.all_kats()


def params_for(over):
    prm = {**cp.GROUND_PARAMS, **cp.PROFILES["simulation"], **over}
    return cp.load_params("simulation", over), prm


def same_f32(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    if a.shape != b.shape:
        return False
    nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(nan | (a.view(np.uint32) == b.view(np.uint32))))


@pytest.mark.parametrize("kat", KATS, ids=[k[0] for k in KATS])
@pytest.mark.parametrize("mode", ["pipeline", "detect"])
def test_kat_oracle_vs_numpy(kat, mode):
    name, pts, over, _ = kat
    params, prm = params_for(over)
    msg = cp.PointCloud2.from_xyzi(pts)
    det, hdr = O.run(params, msg, O.MODE_PIPELINE if mode == "pipeline" else O.MODE_DETECT, O.ORDER_STABLE)
    ref = R.pipeline(pts.copy(), prm, ground=(mode == "pipeline"))
    assert det.n_filtered == ref["M"], name
    assert same_f32(det.voxels, ref["vox"]), name
    assert bool(det.flags & 1) == ref["passthrough"], name
    # cluster sets always; order exactly when <= 16 clusters (stable insertion sort)
    got_sets = sorted(tuple(c) for c in det.clusters)
    assert got_sets == sorted(tuple(c) for c in ref["clusters"]), name
    if len(ref["clusters"]) <= 16:
        assert [list(c) for c in det.clusters] == ref["clusters"], name
        assert same_f32(det.centroids, ref["centroids"]), name


def _run(kat, mode):
    name, pts, over, exp = kat
    params, _ = params_for(over)
    msg = cp.PointCloud2.from_xyzi(pts)
    return O.run(params, msg, mode)


def test_kat_ground_threshold_double_compare():
    g, hdr = _run(KC.kat_ground_threshold(), O.MODE_GROUND)
    kept = g.view(np.float32).reshape(-1, 8)[: int(hdr[1])]
    assert set(np.unique(kept[:, 4]).tolist()) == {2.0}


def test_kat_sector16_is_its_own_bin():
    g, hdr = _run(KC.kat_sector16(), O.MODE_GROUND)
    kept = g.view(np.float32).reshape(-1, 8)[: int(hdr[1])]
    assert {8.0, 9.0} <= set(kept[:, 4].tolist())


@pytest.mark.parametrize("builder,key", [(KC.kat_tolerance, "sizes"), (KC.kat_cluster_sizes, "sizes")])
def test_kat_cluster_sizes(builder, key):
    kat = builder()
    det, _ = _run(kat, O.MODE_DETECT)
    assert [len(c) for c in det.clusters] == kat[3][key]


def test_kat_many_equal_clusters_uses_introsort_order():
    det, _ = _run(KC.kat_many_equal_clusters(), O.MODE_DETECT)
    sizes = [len(c) for c in det.clusters]
    assert len(sizes) >= 17 and sizes == sorted(sizes, reverse=True)


def test_kat_voxel_passthrough():
    det, _ = _run(KC.kat_voxel_passthrough(), O.MODE_DETECT)
    assert det.flags & 1 and len(det.voxels) == det.n_filtered == 4


def test_kat_zero_pad_survives():
    det, _ = _run(KC.kat_zero_pad_survives(), O.MODE_PIPELINE)
    assert det.n_filtered > det.n_kept - 1  # pads joined the filtered cloud
    origin = np.all(det.voxels[:, :3] == 0.0, axis=1)
    assert origin.sum() == 1


def test_kat_empty_and_all_filtered():
    det, hdr = _run(KC.kat_empty(), O.MODE_PIPELINE)
    assert det.n_points == 0 and len(det.voxels) == 0 and len(det.clusters) == 0
    det, hdr = _run(KC.kat_all_filtered(), O.MODE_PIPELINE)
    assert det.n_filtered == 0 and len(det.clusters) == 0
