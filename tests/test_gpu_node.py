"""GPU parity of the detector node after the hot path: the cone re-crop (cg_recrop,
get_reconstructed_cone, src/cone_detection.cpp:222-238) and the whole ConeDetector::cloud_handler
(src/cone_detection.cpp:130-187: hot path, tracking, re-crop, colour service, the four published
clouds) against the CPU restatement, bit for bit.

The colour service is a stand-in that depends on the exact crop (point count and intensity
sum), so a crop that differs in any point usually changes a colour and the published clouds."""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from cones_perception_amd import _abi

pytestmark = pytest.mark.gpu


def _frame(rings=64, cols=1024, frame=0, clutter=20, cpr=6, step=16):
    raw = cp.synth_frames(1, first_frame=frame, rings=rings, cols=cols, clutter=clutter, cones_per_row=cpr,
                          point_step=step)
    return cp.frame_cloud(raw[0], point_step=step)


def _same_crops(got, ref, ctx):
    assert len(got) == len(ref), ctx
    for c, (g, r) in enumerate(zip(got, ref)):
        assert g.shape == r.shape, (ctx, c, g.shape, r.shape)
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), (ctx, c)


def _centres(det, rng, extra=12):
    """The detection's centroids, centres scattered over the cloud, one at the origin (the
    pipeline's zero pads), a NaN and one far away."""
    pts = [det.centroids.reshape(-1, 2), rng.uniform(-9, 9, (extra, 2)),
           [[0.0, 0.0], [np.nan, 1.0], [500.0, 500.0], [0.1, -0.05]]]
    return np.concatenate([np.asarray(p, np.float32).reshape(-1, 2) for p in pts]).astype(np.float32)


@pytest.fixture(scope="module")
def params():
    return cp.load_params("simulation")


@pytest.mark.parametrize("rings,cols", [(64, 1024), (128, 1024)])   # 128 x 1024: the large-frame path
def test_recrop_pipeline_matches_oracle(params, rings, cols):
    msg = _frame(rings, cols, frame=2)
    pipe = cp.ConePipeline(params)
    det = pipe.cloud_handler(msg)
    cen = _centres(det, np.random.default_rng(rings))
    got = pipe.recrop(cen)
    ref = O.recrop(params, msg, O.MODE_PIPELINE, cen)
    _same_crops(got, ref, f"pipeline {rings}x{cols}")
    assert sum(len(c) for c in got) > 0
    assert len(got[-4]) >= det.n_points - det.n_kept   # the origin box holds every zero pad


def test_recrop_detect_matches_oracle(params):
    msg = _frame(frame=3)
    d = cp.ConeDetector(params)
    det = d.cloud_handler(msg)
    cen = _centres(det, np.random.default_rng(5))
    _same_crops(d.recrop(cen), O.recrop(params, msg, O.MODE_DETECT, cen), "detect")


def test_recrop_without_intensity_field_reads_x(params):
    """src/cone_detection.cpp:142-151: no intensity field -> intensity aliases x (offset 0)."""
    msg = _frame(frame=4)
    msg.fields = [f for f in msg.fields if f.name != "intensity"]
    d = cp.ConeDetector(params)
    det = d.cloud_handler(msg)
    cen = _centres(det, np.random.default_rng(6))
    got = d.recrop(cen)
    _same_crops(got, O.recrop(params, msg, O.MODE_DETECT, cen, intensity_offset=0), "no intensity")
    for c in got:
        assert np.array_equal(c[:, 3].view(np.uint32), c[:, 0].view(np.uint32))


def test_recrop_many_centres_and_edges(params):
    """More centres than one launch takes (256), duplicates, and boxes whose edges sit exactly
    on points (the double compares are inclusive)."""
    msg = _frame(frame=5)
    pipe = cp.ConePipeline(params)
    pipe.cloud_handler(msg)
    xyz = msg.xyzi()
    rng = np.random.default_rng(9)
    pick = xyz[rng.integers(0, len(xyz), 300)]
    half = np.float64(np.float32(0.228)) / 1.5
    cen = np.concatenate([pick[:, :2],
                          (pick[:40, :2].astype(np.float64) - half).astype(np.float32),   # edge on a point
                          pick[:10, :2]]).astype(np.float32)
    _same_crops(pipe.recrop(cen), O.recrop(params, msg, O.MODE_PIPELINE, cen), "many")
    assert pipe.recrop(np.zeros((0, 2), np.float32)) == []


def test_recrop_requires_a_detector_call(params):
    h = cp.ConePipeline(params)
    with pytest.raises(_abi.CgError):
        h.recrop([[1.0, 2.0]])


def _service(crop_xyzi):
    return (len(crop_xyzi) + int(np.floor(crop_xyzi[:, 3].astype(np.float64).sum()))) % 4 if len(crop_xyzi) else 0


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("classify,buffer", [(True, False), (True, True), (False, True)])
def test_node_matches_oracle_over_frames(params, fused, classify, buffer):
    """Eight consecutive frames through ConeDetectorNode (GPU) and the restated node fed with the
    restated detections: the published clouds, headers and field lists. The service call fails
    on frames 3 and 6 (every colour then stays unknown)."""
    state = {"frame": 0, "asked": 0}
    failing = {3, 6}

    def classifier(msgs):
        state["asked"] += len(msgs)
        assert all(m.header.get("frame_id") == "cloud" and m.point_step == 32 for m in msgs)
        if state["frame"] in failing:
            return None
        return [_service(m.xyzi()) for m in msgs if m.width]   # the server skips empty crops

    node = cp.ConeDetectorNode(params, classify_colors=classify, use_points_buffer=buffer, classifier=classifier,
                               fused_ground_removal=fused)
    ref_node = O.Node(classify, buffer, params.cones_matching_dist_theshold)
    mode = O.MODE_PIPELINE if fused else O.MODE_DETECT
    published = 0
    base = _frame(frame=10).xyzi()
    rng = np.random.default_rng(11)
    for f in range(8):
        state["frame"] = f
        # one scene seen from a vehicle creeping forward: consecutive frames track
        pts = base.copy()
        pts[:, 0] -= np.float32(0.07 * f)
        pts[:, :3] += rng.normal(0, 0.01, (len(pts), 3)).astype(np.float32)
        msg = cp.PointCloud2.from_xyzi(pts, layout=16)
        msg.header = {"seq": f, "stamp_sec": 100 + f, "stamp_nsec": 123456789, "frame_id": "lidar"}
        outs = node.cloud_handler(msg)
        det, _ = O.run(params, msg, mode)
        ref = ref_node.step(params, msg, mode, det.centroids,
                            lambda crops: None if f in failing else O.server(crops, _service))
        assert len(outs) == 4
        for i, m in enumerate(outs):
            assert m.header == msg.header                                          # line 182
            assert [(q.name, q.offset) for q in m.fields] == [(q.name, q.offset) for q in msg.fields]   # 183
            assert m.point_step == 32 and m.height == 1 and m.width == len(ref[i])
            recs = m.data.view(np.float32).reshape(-1, 8)
            assert np.array_equal(recs[:, 0:2].view(np.uint32), ref[i].view(np.uint32)), (f, i)
            assert np.all(recs[:, 2] == 0) and np.all(recs[:, 3] == 1.0) and np.all(recs[:, 4] == 0)
            published += m.width
    assert published > 0
    assert (state["asked"] > 0) == classify


def _ring_and_cone():
    """A ring of 16 points (radius 0.35 m around (5, 0)): one cluster whose pushed centroid
    (5.05, 0) has no point within the re-crop box (half-width 0.228 / 1.5 m), so its crop is
    empty; and a 6-point cone at (7, 1), a smaller cluster, so it is classified second."""
    a = np.arange(16) * (2 * np.pi / 16)
    ring = np.stack([5 + 0.35 * np.cos(a), 0.35 * np.sin(a), np.zeros(16), np.full(16, 40.0)], 1)
    cone = np.array([[7.0, 1.0, 0.0], [7.05, 1.0, 0.1], [7.0, 1.05, 0.2], [6.95, 1.0, 0.1],
                     [7.0, 0.95, 0.2], [7.02, 1.02, 0.3]])
    cone = np.concatenate([cone, np.full((6, 1), 70.0)], 1)
    return cp.PointCloud2.from_xyzi(np.concatenate([ring, cone]).astype(np.float32), layout=16)


def test_node_short_colour_response_is_positional(params):
    """The reference's server answers only non-empty crops (scripts/color_classifier_server.py:
    83-84) and the node writes the response over colors(n_need, Unknown) from the front
    (src/cone_detection.cpp:328,357-358). With the ring's empty crop first in the request, the
    cone's colour lands on the ring's centroid and the cone stays unknown; GPU node = oracle."""
    msg = _ring_and_cone()
    requests = []

    def classifier(msgs):
        requests.append([m.width for m in msgs])
        return [3 for m in msgs if m.width]

    node = cp.ConeDetectorNode(params, classify_colors=True, use_points_buffer=False, classifier=classifier)
    ref_node = O.Node(True, False, params.cones_matching_dist_theshold)
    for f in range(2):
        outs = node.cloud_handler(msg)
        det, _ = O.run(params, msg, O.MODE_DETECT)
        assert len(det.centroids) == 2
        ref = ref_node.step(params, msg, O.MODE_DETECT, det.centroids, lambda crops: O.server(crops, lambda c: 3))
        for i, m in enumerate(outs):
            got = m.data.view(np.float32).reshape(-1, 8)[:, 0:2]
            assert np.array_equal(got.view(np.uint32), ref[i].view(np.uint32)), (f, i)
    assert requests == [[0, 6]]
    ring_c, cone_c = det.centroids
    assert ref[3].tolist() == [ring_c.tolist()] and ref[0].tolist() == [cone_c.tolist()]


def test_ground_node_message_header_and_fields(params):
    """src/ground_removal.cpp:81-86: header and fields are set before toROSMsg, which replaces
    them: PointXYZI's fields and the input header after PCL's microsecond stamp."""
    msg = _frame(frame=6)
    msg.header = {"seq": 7, "stamp_sec": 1700000000, "stamp_nsec": 987654321, "frame_id": "velodyne"}
    out = cp.GroundRemover(params).cloud_handler(msg)
    assert out.header == {"seq": 7, "stamp_sec": 1700000000, "stamp_nsec": 987654000, "frame_id": "velodyne"}
    assert [(f.name, f.offset) for f in out.fields] == [("x", 0), ("y", 4), ("z", 8), ("intensity", 16)]
    assert (out.point_step, out.width * out.height) == (32, msg.width * msg.height)


def test_handles_leave_no_sticky_hip_error(params):
    """Every handle kind, on a fused-path and a large-path frame, with a re-crop where it applies,
    then closed: the runtime's last-error state stays clean (a stale error would surface in the
    next handle's first launch check)."""
    import ctypes
    cp.lib()
    hip = ctypes.CDLL("libamdhip64.so.7")        # the runtime already loaded (same soname)
    hip.hipGetLastError.restype = ctypes.c_int
    assert hip.hipGetLastError() == 0
    for cls in (cp.ConePipeline, cp.ConeDetector, cp.GroundRemover):
        for rings in (64, 128):
            h = cls(params)
            h.cloud_handler(_frame(rings, 1024, frame=7))
            if cls is not cp.GroundRemover:
                h.recrop([[2.0, 1.0], [0.0, 0.0]])
            h.close()
            assert hip.hipGetLastError() == 0, (cls.__name__, rings)


def test_cpp_node_mirror_demo():
    """host/nodes_demo.cpp: the C++ mirror's two-node chain equals the fused call (hot path), and
    its ConeDetectorNode over a tracked sequence publishes the same clouds either way."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(_abi.LIB_PATH), "nodes_demo")
    import tempfile
    import numpy as np
    wpath = os.path.join(tempfile.mkdtemp(), "dam_net.f32")
    np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dam_net_weights.npy")).astype(
        "<f4").tofile(wpath)
    r = subprocess.run([exe, "5", wpath], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("node frame")]
    assert len(lines) == 5 and all("fused == two-node" in l for l in lines)
    assert any(" unknown=0" not in l or " yellow=0" not in l for l in lines[1:])   # something published
    # the GPU colour classifier (ColorClassifier, cg_classify_colors) as the node's service
    gl = [l for l in r.stdout.splitlines() if l.startswith("gpu colour service frame")]
    assert len(gl) == 5


@pytest.mark.parametrize("mode,rings", [("pipeline", 64), ("detect", 64), ("pipeline", 128)])
def test_batch_recrop_matches_oracle(params, mode, rings):
    """cg_batch_recrop: the re-crop of any frame of a device-resident batch (frames of the
    batch engine, 128-ring frames through the large path) equals the oracle's on that frame."""
    import torch
    F, cols = 3, 1024
    raw = cp.synth_frames(F, first_frame=5, rings=rings, cols=cols, clutter=20, cones_per_row=6)
    d = torch.from_numpy(raw).to(torch.device("cuda", 0))
    eng = cp.BatchEngine(params, device=0)
    m = _abi.CG_MODE_PIPELINE if mode == "pipeline" else _abi.CG_MODE_DETECT
    eng.run(d.data_ptr(), F, rings * cols, 16, mode=m)
    om = O.MODE_PIPELINE if mode == "pipeline" else O.MODE_DETECT
    for f in (F - 1, 0):
        det = eng.fetch(f)
        cen = _centres(det, np.random.default_rng(f))
        got = eng.recrop(f, cen)
        ref = O.recrop(params, cp.frame_cloud(raw[f]), om, cen)
        _same_crops(got, ref, f"batch {mode} frame {f}")
        assert sum(len(c) for c in got) > 0


@pytest.mark.gpu
def test_batch_recrop_refused_after_single_frame_call(params):
    """A single-frame call on a batch engine's handle rewrites frame 0's result slots, so a
    cg_batch_recrop of the earlier batch must fail (CG_E_INVALID), not crop with mixed state."""
    import ctypes
    import torch
    raw = cp.synth_frames(2, first_frame=9, rings=64, cols=1024)
    d = torch.from_numpy(raw).to(torch.device("cuda", 0))
    eng = cp.BatchEngine(params, device=0)
    eng.run(d.data_ptr(), 2, 64 * 1024, 16)
    cen = _centres(eng.fetch(0), np.random.default_rng(3))
    eng.recrop(0, cen)   # valid right after the batch
    msg = cp.frame_cloud(raw[1])   # keeps the bytes the view points at alive
    v = msg.view(intensity_offset=12)
    r = _abi.cg_detect_result()
    _abi.check(cp.lib().cg_pipeline(eng.handle, ctypes.byref(v), ctypes.byref(r)))
    with pytest.raises(_abi.CgError):
        eng.recrop(0, cen)
    eng.run(d.data_ptr(), 2, 64 * 1024, 16)   # a new batch makes it valid again
    got = eng.recrop(1, cen)
    _same_crops(got, O.recrop(params, cp.frame_cloud(raw[1]), O.MODE_PIPELINE, cen), "after re-run")
