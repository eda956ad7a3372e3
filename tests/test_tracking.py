"""Tracking and colour clouds (ConeDetector::get_centroid_clouds, src/cone_detection.cpp:251-339):
the C-ABI tracker (host code, no GPU) against the CPU restatement over random multi-frame
centroid sequences, for every combination of classify_colors / use_points_buffer, with failed
colour-service calls and matches exactly at the threshold.

The colour service stands in as a deterministic answer sequence: the k-th classification of
the run gets colour k*7+3 mod 4, so both sides must ask for the same cones in the same order.
Crops are not compared here (the whole cloud is empty; tests/test_gpu_node.py covers them)."""
import itertools

import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from cones_perception_amd import _abi


def _sequences(seed, frames=40):
    """Cones at fixed places, each frame a random subset with jitter up to 0.6 m (threshold 0.5),
    plus a few centroids placed at exactly 0.5 m / one float step inside it from a previous
    one. Order shuffled per frame (cluster order)."""
    rng = np.random.default_rng(seed)
    base = rng.uniform(-8, 8, (14, 2)).astype(np.float32)
    out = []
    prev = None
    for f in range(frames):
        keep = rng.random(base.shape[0]) < 0.7
        cen = base[keep] + rng.normal(0, 0.25, (int(keep.sum()), 2)).astype(np.float32)
        if prev is not None and len(prev) and f % 3 == 0:
            q = prev[0]
            edge = np.array([[q[0] + np.float32(0.5), q[1]],
                             [np.nextafter(q[0] + np.float32(0.5), np.float32(-np.inf)), q[1]],
                             [q[0], q[1] - np.float32(0.5)]], np.float32)
            cen = np.concatenate([cen, edge])
        cen = cen[rng.permutation(len(cen))].astype(np.float32)
        if f % 11 == 5:
            cen = cen[:0]                                  # a frame without cones
        out.append(cen)
        prev = cen
    return out


def _run_product(seq, classify, buffer, fail):
    t = cp.ConeTracker(classify, buffer, 0.5)
    k = 0
    clouds = []
    for f, cen in enumerate(seq):
        st, need = t.match(cen)
        assert st.shape == (len(cen),) and need == int((st == _abi.CG_TRACK_NEED_COLOR).sum())
        colours = None
        if need and f not in fail:
            colours = [(kk * 7 + 3) % 4 for kk in range(k, k + need)]
            k += need
        t.commit(colours)
        clouds.append(t.clouds())
    return clouds


def _run_oracle(seq, classify, buffer, fail):
    params = cp.load_params("simulation")
    empty = cp.PointCloud2.from_xyzi(np.zeros((0, 4), np.float32))
    node = O.Node(classify, buffer, 0.5)
    state = {"k": 0}
    clouds = []
    for f, cen in enumerate(seq):
        asked = []

        def service(_crop):
            if f in fail:
                return -1
            asked.append(1)
            return ((state["k"] + len(asked) - 1) * 7 + 3) % 4

        clouds.append(node.step(params, empty, O.MODE_DETECT, cen, service))
        state["k"] += len(asked)
    return clouds


@pytest.mark.parametrize("classify,buffer", list(itertools.product([True, False], [True, False])))
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tracker_matches_restatement(classify, buffer, seed):
    seq = _sequences(seed)
    fail = {7, 19} if classify else set()
    got = _run_product(seq, classify, buffer, fail)
    ref = _run_oracle(seq, classify, buffer, fail)
    published = 0
    for f, (g, r) in enumerate(zip(got, ref)):
        for i in range(4):
            assert np.array_equal(g[i].view(np.uint32), r[i].view(np.uint32)), (f, i, g[i], r[i])
            published += len(g[i])
    assert published > 0


def test_first_frame_publishes_nothing():
    t = cp.ConeTracker(False, False)
    st, need = t.match([[3.0, 1.0], [4.0, -1.0]])
    assert list(st) == [_abi.CG_TRACK_DROPPED] * 2 and need == 0
    t.commit()
    assert all(len(c) == 0 for c in t.clouds())
    st, _ = t.match([[30.0, 1.0]])                       # buffer off: any previous cone publishes
    assert list(st) == [cp.UNKNOWN]


def test_commit_validates_colours():
    t = cp.ConeTracker(True, False)
    t.match([[1.0, 1.0]]); t.commit()
    _, need = t.match([[1.0, 1.0], [2.0, 2.0]])
    assert need == 2
    with pytest.raises(_abi.CgError):
        t.commit([1])                                      # one colour per cone that needs one
    with pytest.raises(_abi.CgError):
        t.commit([1, 4])                                   # out of range
    t.commit([cp.BLUE, cp.ORANGE])
    c = t.clouds()
    assert len(c[cp.BLUE]) == 1 and len(c[cp.ORANGE]) == 1
    st, need = t.match([[1.0, 1.05], [2.0, 2.0], [5.0, 5.0]])   # colours known from last frame
    assert list(st) == [cp.BLUE, cp.ORANGE, _abi.CG_TRACK_NEED_COLOR] and need == 1
