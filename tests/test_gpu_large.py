"""GPU parity of the large-frame path (cg_large.hip): frames of more than 65,536 points, and
every frame forced through it (cg_debug_route), against the CPU restatement bit for bit.

Route 1 sends a frame through the multi-workgroup front (pass 1 / decide per 64k chunk);
route 2 also forces the global HBM backend (radix-sorted voxel keys, neighbour-grid
union-find, CSR by sort) where the LDS backend would normally serve. Both must reproduce the
frame kernel's results exactly, so the small synthetic frames and the known-answer clouds
check the large path's edge semantics at sizes the oracle finishes in milliseconds.
"""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import assert_same_detection, same_bits
from kat_clouds import all_kats

pytestmark = pytest.mark.gpu


def _same_ground(out, ref, hdr, ctx):
    """Declared fields x, y, z, data[3], intensity; PCL's padding bytes are undefined."""
    assert out.n_kept == int(hdr[1]), ctx
    g = out.data.view(np.float32).reshape(-1, 8)
    r = ref.view(np.float32).reshape(-1, 8)
    assert np.array_equal(g[:, :5].view(np.uint32), r[:, :5].view(np.uint32)), ctx


@pytest.fixture(scope="module")
def params():
    return cp.load_params("simulation")


def _frame(rings, cols, frame=0, clutter=0, cpr=5):
    raw = cp.synth_frames(1, first_frame=frame, rings=rings, cols=cols, clutter=clutter, cones_per_row=cpr)
    return cp.frame_cloud(raw[0])


@pytest.mark.parametrize("rings,cols", [(128, 1024), (96, 1024), (65, 1024)])
def test_large_pipeline_matches_oracle(params, rings, cols):
    msg = _frame(rings, cols, frame=3)
    got = cp.ConePipeline(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    assert got.n_points == rings * cols
    assert_same_detection(got, ref, f"{rings}x{cols}")


@pytest.mark.parametrize("rings,cols", [(128, 1024), (96, 1024)])
def test_large_detector_matches_oracle(params, rings, cols):
    msg = _frame(rings, cols, frame=5)
    got = cp.ConeDetector(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_DETECT)
    assert_same_detection(got, ref, f"detect {rings}x{cols}")


@pytest.mark.parametrize("rings,cols", [(128, 1024), (96, 1000)])
def test_large_ground_removal_matches_oracle(params, rings, cols):
    msg = _frame(rings, cols, frame=7)
    out = cp.GroundRemover(params).cloud_handler(msg)
    ref, hdr = O.run(params, msg, O.MODE_GROUND)
    _same_ground(out, ref, hdr, f"{rings}x{cols}")


def test_large_batch_two_frames(params):
    import torch
    rings, cols = 128, 1024
    raw = cp.synth_frames(2, first_frame=11, rings=rings, cols=cols)
    eng = cp.BatchEngine(params)
    d = torch.from_numpy(raw).cuda()
    eng.run(d.data_ptr(), 2, rings * cols, 16)
    for f in range(2):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE)
        assert_same_detection(eng.fetch(f), ref, f"batch frame {f}")


@pytest.mark.parametrize("route", [1, 2])
@pytest.mark.parametrize("frame", [0, 1])
def test_forced_route_matches_oracle(params, route, frame):
    msg = _frame(64, 1024, frame=frame)
    got = cp.ConePipeline(params).debug_route(route).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    assert_same_detection(got, ref, f"route {route}")


@pytest.mark.parametrize("route", [0, 2])
def test_large_passthrough_frame(route):
    """PCL's overflow guard on a large frame (points 1 km up; the distance filter opened so they
    and the far wall reach the voxel grid): the voxel cloud is the detector input in point order,
    unsorted, through the device-sized backend (route 0) and the host-sized one (route 2)."""
    params = cp.load_params("simulation", {"distance_treshold_max": 1e5})
    raw = cp.synth_frames(1, first_frame=4, rings=128, cols=1024, clutter=40, cones_per_row=10)
    pts = raw[0].view(np.float32).reshape(-1, 4)
    pts[5::20011, 2] = 1000.0
    msg = cp.frame_cloud(raw[0])
    got = cp.ConePipeline(params).debug_route(route).cloud_handler(msg)
    ref, hdr = O.run(params, msg, O.MODE_PIPELINE)
    assert got.flags & cp.CG_F_VOXEL_PASSTHROUGH and int(hdr[2]) > 4096
    assert_same_detection(got, ref, f"passthrough route {route}")


@pytest.mark.parametrize("route", [1, 2])
def test_forced_route_dense_frame(params, route):
    msg = _frame(64, 1024, frame=2, clutter=40, cpr=10)
    got = cp.ConePipeline(params).debug_route(route).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    assert_same_detection(got, ref, f"dense route {route}")


@pytest.mark.parametrize("route", [1, 2])
@pytest.mark.parametrize("mode", ["pipeline", "detect", "ground"])
@pytest.mark.parametrize("kat", all_kats(), ids=lambda k: k[0])
def test_forced_route_kats(kat, mode, route):
    name, pts, over, _ = kat
    params = cp.load_params("simulation", over)
    msg = cp.PointCloud2.from_xyzi(pts)
    if mode == "ground":
        out = cp.GroundRemover(params).debug_route(route).cloud_handler(msg)
        ref, hdr = O.run(params, msg, O.MODE_GROUND)
        _same_ground(out, ref, hdr, name)
        return
    cls = cp.ConePipeline if mode == "pipeline" else cp.ConeDetector
    got = cls(params).debug_route(route).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE if mode == "pipeline" else O.MODE_DETECT)
    assert_same_detection(got, ref, f"{name} {mode} route {route}")


def test_c5_dense_million_point_frame(params):
    """C5's frame shape: 128 rings x 8192 columns = 1,048,576 points with dense clutter."""
    msg = _frame(128, 8192, frame=0, clutter=60, cpr=12)
    got = cp.ConePipeline(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    assert got.n_points == 1 << 20
    assert got.voxels.shape[0] > 1024          # the global backend ran
    assert_same_detection(got, ref, "C5")


def test_c5_frame_through_detector(params):
    """The detector alone on C5's frame: ~550k filtered points reach the voxel stage, so the
    single-pass scan over them spans ~135 tiles and each tile's look-back crosses more than
    one 64-tile window."""
    msg = _frame(128, 8192, frame=0, clutter=60, cpr=12)
    got = cp.ConeDetector(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_DETECT)
    assert ref.n_filtered > 64 * 4096
    assert_same_detection(got, ref, "C5 detect")


@pytest.mark.parametrize("rings,cols,clutter", [(128, 4096, 60), (128, 8192, 60)])
def test_pcl_sort_leaves_in_hbm(params, rings, cols, clutter):
    """cg_debug_route 5: the PCL voxel sort stops after one partition level, so both halves of
    the index_vector (longer than the 4,096-record LDS leaf) are finished in HBM by two
    workgroups side by side, each in its own span of the scratch arrays (the span boundary is
    where round 2 found a neighbour's word overwritten)."""
    msg = _frame(rings, cols, frame=1, clutter=clutter, cpr=12)
    pipe = cp.ConePipeline(params)
    pipe.debug_route(5)
    got = pipe.cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    assert got.n_filtered > 2 * 4096
    assert_same_detection(got, ref, f"route 5 {rings}x{cols}")


def test_pcl_sort_hbm_leaves_beyond_16_bit_counts(params):
    """cg_debug_route 5 on the detector's C5 frame (~550k filtered points): one partition level
    leaves two halves of ~275k records, each finished in HBM by one workgroup. Past 65,535
    records the >= / <= pivot counts no longer fit two 16-bit halves of one scan word; the HBM
    form scans them separately there (cg_pcl.h pcl_sort), so the order stays std::sort's."""
    msg = _frame(128, 8192, frame=0, clutter=60, cpr=12)
    det = cp.ConeDetector(params)
    det.debug_route(5)
    got = det.cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_DETECT)
    assert ref.n_filtered > 2 * 65536 + 4096
    assert_same_detection(got, ref, "C5 detect route 5")
    det.debug_route(0)    # the route cleared: the next frame takes every partition level again
    got = det.cloud_handler(msg)
    assert_same_detection(got, ref, "C5 detect after route 5")


@pytest.mark.parametrize("mode", ["pipeline", "detect"])
def test_large_batch_pipelined_over_two_scratch_sets(params, mode):
    """Several large frames in one batch: frame f + 1's front runs on the second scratch set
    while the host sizes frame f's backend (cg_run_large); every frame bit-exact, in both the
    LDS and the global backend."""
    import torch
    raw = np.concatenate([cp.synth_frames(1, first_frame=20 + f, rings=128, cols=1024, clutter=c, cones_per_row=8)
                          for f, c in enumerate((0, 60, 0, 200, 20))])
    eng = cp.BatchEngine(params)
    d = torch.from_numpy(raw).cuda()
    m = cp.CG_MODE_PIPELINE if mode == "pipeline" else cp.CG_MODE_DETECT
    for rep in range(2):   # the sets are reused by the next batch
        eng.run(d.data_ptr(), raw.shape[0], 128 * 1024, 16, mode=m)
        for f in range(raw.shape[0]):
            ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE if mode == "pipeline" else O.MODE_DETECT)
            assert_same_detection(eng.fetch(f), ref, f"pipelined batch {rep} frame {f}")


def test_hint_sequence_small_large_medium(params):
    """The device-sized path leaves the LDS backend's launch out after a large frame (the
    pinned hint word). One handle runs frames whose sizes jump both ways (a small frame after a
    large one takes the global backend) and every frame must stay bit-exact."""
    seq = [_frame(128, 1024, frame=3),                          # small: the LDS backend
           _frame(128, 8192, frame=0, clutter=60, cpr=12),      # C5: every partition level
           _frame(128, 1024, frame=3),                          # small after large: global backend
           _frame(128, 8192, frame=0, clutter=60, cpr=12),      # large after small
           _frame(128, 2048, frame=6, clutter=20, cpr=8),       # medium
           _frame(128, 8192, frame=1, clutter=60, cpr=12)]      # large after medium
    pipe = cp.ConePipeline(params)
    ms = []
    for i, msg in enumerate(seq):
        got = pipe.cloud_handler(msg)
        ref, hdr = O.run(params, msg, O.MODE_PIPELINE)
        ms.append(int(hdr[2]))
        assert_same_detection(got, ref, f"sequence frame {i} (M {ms[-1]})")
    assert ms[0] <= 1024 and ms[1] > 8 * 4096, ms


def test_graph_cache_rotating_buffers(params):
    """The device-sized path keys one captured graph per (arguments, frame): a caller rotating
    more input buffers than the cache holds (32) evicts the least recently used graph and
    captures again; every frame stays bit-exact, including buffers whose graph was evicted."""
    import torch
    raw = cp.synth_frames(1, first_frame=4, rings=128, cols=1024, clutter=0, cones_per_row=8)
    n = 128 * 1024
    ref, _ = O.run(params, cp.frame_cloud(raw[0]), O.MODE_PIPELINE)
    copies = 36
    d = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(raw, (copies,) + raw.shape[1:]))).cuda()
    eng = cp.BatchEngine(params)
    for rep in range(2):
        for k in list(range(copies)) + [0, 1, 35]:
            eng.run(d[k].data_ptr(), 1, n, 16, mode=cp.CG_MODE_PIPELINE)
            assert_same_detection(eng.fetch(0), ref, f"rotation {rep} buffer {k}")


@pytest.mark.parametrize("rings,cols", [(256, 16384), (257, 16384)])
def test_largest_device_sized_frame(params, rings, cols):
    """The device-sized path's largest frame (LG_DEV_MAX_POINTS = 4,194,304 points: 1,024 chunks
    taken by ticket in lg_decide_write, their look-back and fold) and one ring more, which takes
    the host-sized path; both bit-exact. (The 4M frame's 7,510 voxels also put lg_cluster_tail on
    its HBM form, past LG_TAIL_LDS.)"""
    msg = _frame(rings, cols, frame=2, clutter=60, cpr=12)
    got = cp.ConePipeline(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    assert got.n_points == rings * cols
    assert_same_detection(got, ref, f"{rings}x{cols}")


def test_device_wait_timeout_fails_loudly(params):
    """A large frame whose device-side wait gives up (LG_PQ_TIMEOUT; forced by cg_debug_route 10
    at its first partition level) fails its fetch with CG_E_DEVICE instead of returning void
    results; the handle serves the next frame exactly."""
    msg = _frame(128, 4096, frame=5, clutter=60, cpr=12)   # (M past the LDS backend: the levels run)
    ref, hdr = O.run(params, msg, O.MODE_PIPELINE)
    assert int(hdr[2]) > 4096
    pipe = cp.ConePipeline(params)
    pipe.debug_route(10)
    with pytest.raises(Exception, match="gave up"):
        pipe.cloud_handler(msg)
    pipe.debug_route(0)
    assert_same_detection(pipe.cloud_handler(msg), ref, "after the failed frame")
