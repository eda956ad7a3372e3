"""Tracking and colour clouds (ConeDetector::get_centroid_clouds, src/cone_detection.cpp:251-339):
the C-ABI tracker (host code, no GPU) against the CPU restatement over random multi-frame
centroid sequences, for every combination of classify_colors / use_points_buffer, with failed
colour-service calls, short service responses (the reference's server skips empty crops,
scripts/color_classifier_server.py:83-84, and the node applies the response positionally,
src/cone_detection.cpp:328,357-358) and matches exactly at the threshold.

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


def _answers(k, need, f, short):
    """The service's response: one colour per request entry, or only the first half of them on
    the `short` frames (as when the server skipped empty crops)."""
    n = (need + 1) // 2 if f in short else need
    return [(kk * 7 + 3) % 4 for kk in range(k, k + n)]


def _run_product(seq, classify, buffer, fail, short=()):
    t = cp.ConeTracker(classify, buffer, 0.5)
    k = 0
    clouds = []
    for f, cen in enumerate(seq):
        st, need = t.match(cen)
        assert st.shape == (len(cen),) and need == int((st == _abi.CG_TRACK_NEED_COLOR).sum())
        colours = None
        if need and f not in fail:
            colours = _answers(k, need, f, short)
            k += need
        t.commit(colours)
        clouds.append(t.clouds())
    return clouds


def _run_oracle(seq, classify, buffer, fail, short=()):
    params = cp.load_params("simulation")
    empty = cp.PointCloud2.from_xyzi(np.zeros((0, 4), np.float32))
    node = O.Node(classify, buffer, 0.5)
    state = {"k": 0}
    clouds = []
    for f, cen in enumerate(seq):
        def service(crops):
            if f in fail:
                return None
            r = _answers(state["k"], len(crops), f, short)
            state["k"] += len(crops)
            return r

        clouds.append(node.step(params, empty, O.MODE_DETECT, cen, service))
    return clouds


@pytest.mark.parametrize("classify,buffer", list(itertools.product([True, False], [True, False])))
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tracker_matches_restatement(classify, buffer, seed):
    seq = _sequences(seed)
    fail = {7, 19} if classify else set()
    short = {4, 9, 13, 22, 30} if classify else set()
    got = _run_product(seq, classify, buffer, fail, short)
    ref = _run_oracle(seq, classify, buffer, fail, short)
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
        t.commit([1, 2, 3])                                # more colours than cones that need one
    with pytest.raises(_abi.CgError):
        t.commit([1, 4])                                   # out of range
    t.commit([cp.BLUE, cp.ORANGE])
    c = t.clouds()
    assert len(c[cp.BLUE]) == 1 and len(c[cp.ORANGE]) == 1
    st, need = t.match([[1.0, 1.05], [2.0, 2.0], [5.0, 5.0]])   # colours known from last frame
    assert list(st) == [cp.BLUE, cp.ORANGE, _abi.CG_TRACK_NEED_COLOR] and need == 1


def test_short_response_is_positional():
    """A response of L < n_need colours colours the first L cones that need one, in request
    order; the rest stay unknown (src/cone_detection.cpp:328,357-358). A response longer than
    the request is refused (the reference would write past its colour vector)."""
    t = cp.ConeTracker(True, False)
    t.match([[3.0, 1.0], [4.0, -1.0], [6.0, 2.0]])
    t.commit()
    st, need = t.match([[3.0, 1.0], [4.0, -1.0], [6.0, 2.0]])
    assert need == 3
    t.commit([2])
    c = t.clouds()
    assert c[2].tolist() == [[3.0, 1.0]] and c[0].tolist() == [[4.0, -1.0], [6.0, 2.0]]
    t.match([[9.0, 9.0]])
    with pytest.raises(RuntimeError):
        t.commit([1, 2])
