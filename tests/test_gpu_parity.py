"""GPU parity: the HIP path (through the C-ABI) against the CPU restatement, bit for bit.

Integer/index outputs (K, M, V, C, cluster index sets, labels) must be identical, and every
float output (voxel centroids, cluster centroids) bit-identical: the device restates the
reference's float/double arithmetic exactly (cg_math.h) and sums each voxel in PCL's std::sort
permutation of index_vector (the default CG_VOXEL_ORDER_PCL), compared with the oracle's
ORDER_PCL mode (tests/oracle_py.py's default). The north star's 1e-5 m centroid tolerance is
therefore met with 0 error. Sizes: C1 (16 rings x 1024) and C2 (64 x 1024) synthetic frames.
"""
import ctypes as C

import numpy as np
import pytest

import cones_perception_amd as cp
from cones_perception_amd import _abi
import oracle_py as O
from helpers import assert_same_detection

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def params():
    return cp.load_params("simulation")


@pytest.fixture(scope="module")
def pipe(params):
    return cp.ConePipeline(params)


@pytest.fixture(scope="module")
def det(params):
    return cp.ConeDetector(params)


@pytest.fixture(scope="module")
def ground(params):
    return cp.GroundRemover(params)


def test_atan2f_device_matches_host_libm(pipe):
    rng = np.random.default_rng(7)
    n = 1 << 22
    y = rng.standard_normal(n).astype(np.float32) * np.float32(10)
    x = rng.standard_normal(n).astype(np.float32) * np.float32(10)
    # raw bit patterns (incl. inf/nan/denormals), axis points and sector boundaries
    y[:65536] = rng.integers(0, 2**32, 65536, dtype=np.uint64).astype(np.uint32).view(np.float32)
    x[:65536] = rng.integers(0, 2**32, 65536, dtype=np.uint64).astype(np.uint32).view(np.float32)
    # sector boundaries (within the approximation error and across the certificate margins)
    # and the angle-filter threshold +-1.3 of the self-test kernel
    ang = np.concatenate([np.arange(17, dtype=np.float64) * 22.0 * np.pi / 180.0, [1.3, -1.3]])
    k = np.concatenate([np.repeat(ang, 4096) + rng.uniform(-3e-6, 3e-6, ang.size * 4096),
                        np.repeat(ang, 2048) + rng.uniform(-8e-5, 8e-5, ang.size * 2048)])
    rad = rng.uniform(0.5, 60.0, k.size)
    x[65536:65536 + k.size] = (np.cos(k) * rad).astype(np.float32)
    y[65536:65536 + k.size] = (np.sin(k) * rad).astype(np.float32)
    out = np.zeros(2 * n, np.float32)
    _abi.check(_abi.lib().cg_selftest_atan2f(pipe.handle, y.ctypes.data, x.ctypes.data, out.ctypes.data, n))
    ol = O.lib()
    sample = np.concatenate([np.arange(0, 65536 + k.size), rng.integers(0, n, 200000)])
    bad = []
    for i in sample:
        a = ol.oracle_atan2f(float(y[i]), float(x[i]))
        g = out[2 * i]
        if not (np.float32(a).view(np.uint32) == np.float32(g).view(np.uint32) or (np.isnan(a) and np.isnan(g))):
            bad.append((int(i), "atan2f", float(a), float(g)))
        elif not np.isnan(a):
            a32 = np.float32(a)
            rm = bool(a32 <= np.float32(-1.3) or a32 >= np.float32(1.3))
            want = ol.oracle_sector(float(y[i]), float(x[i])) + (32 if rm else 0)
            if int(out[2 * i + 1]) != want:
                bad.append((int(i), "class", float(a), float(x[i]), float(y[i]), want, int(out[2 * i + 1])))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:6]}"


def test_sqrt_device_correctly_rounded(pipe):
    rng = np.random.default_rng(3)
    n = 1 << 20
    s = np.abs(rng.standard_normal(n)) * 10.0 ** rng.uniform(-6, 6, n)
    out = np.zeros(n)
    _abi.check(_abi.lib().cg_selftest_sqrt(pipe.handle, s.ctypes.data, out.ctypes.data, n))
    assert np.array_equal(out.view(np.uint64), np.sqrt(s).view(np.uint64))


@pytest.mark.parametrize("rings,cols,frame", [(16, 1024, 0), (16, 1024, 1), (64, 1024, 0), (64, 1024, 5),
                                              (64, 1024, 17)])
def test_pipeline_matches_oracle(params, pipe, rings, cols, frame):
    raw = cp.synth_frames(1, first_frame=frame, rings=rings, cols=cols)
    msg = cp.frame_cloud(raw[0])
    got = pipe.cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE)
    assert ref.cluster_offsets.size > 1
    assert_same_detection(got, ref, f"pipeline {rings}x{cols} f{frame}")


def test_single_frame_staging_grows_and_shrinks(params):
    """One fresh handle, frames whose sizes grow and shrink the pinned staging buffer between
    calls: each chunk workgroup waits for its chunk's publish word, which the host stores after
    copying the chunk (after the launch). The round-3 fault was the publish words freed with a
    growing staging buffer (a 16k frame, then a 64k one)."""
    pipe = cp.ConePipeline(params)
    for rings, cols, frame in [(1, 100, 0), (16, 1024, 1), (64, 1024, 2), (3, 1000, 3), (64, 1024, 4),
                               (8, 1000, 5)]:
        raw = cp.synth_frames(1, first_frame=frame, rings=rings, cols=cols)
        msg = cp.frame_cloud(raw[0])
        got = pipe.cloud_handler(msg)
        ref, _ = O.run(params, msg, O.MODE_PIPELINE)
        assert_same_detection(got, ref, f"staged {rings}x{cols} f{frame}")


def test_single_frame_done_word_never_stale(params):
    """The split launch packs its results into pinned host memory and then stores a done word
    the host polls: every packed word must be visible before the word. Frames with different
    results alternate for 300 calls on one handle; a result read before its pack landed would
    carry the previous frame's counts or centroids."""
    pipe = cp.ConePipeline(params)
    frames = []
    for f, clutter, cpr in ((0, 0, 5), (1, 60, 9), (2, 20, 3)):
        msg = cp.frame_cloud(cp.synth_frames(1, first_frame=f, rings=64, cols=1024, clutter=clutter,
                                             cones_per_row=cpr)[0])
        frames.append((msg, O.run(params, msg, O.MODE_PIPELINE)[0]))
    assert len({r.voxels.shape[0] for _, r in frames}) == 3   # distinguishable results
    for i in range(300):
        msg, ref = frames[i % 3]
        assert_same_detection(pipe.cloud_handler(msg), ref, f"call {i}")


def test_batch_fetch_between_single_frames(params):
    """A batch run and a batch fetch on the handle between single-frame calls: the fetch copies
    the device pack buffer to the pinned one, but never its done word (the split launch's
    sequence word, which the next single-frame call polls). Every single frame and every fetched
    batch frame against the oracle."""
    import torch
    pipe = cp.ConePipeline(params)
    frames = []
    for f, clutter, cpr in ((4, 0, 5), (5, 40, 8), (6, 10, 3)):
        msg = cp.frame_cloud(cp.synth_frames(1, first_frame=f, rings=64, cols=1024, clutter=clutter,
                                             cones_per_row=cpr)[0])
        frames.append((msg, O.run(params, msg, O.MODE_PIPELINE)[0]))
    raw = cp.synth_frames(2, first_frame=40, rings=64, cols=1024, clutter=20, cones_per_row=6)
    brefs = [O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE)[0] for f in range(2)]
    d = torch.from_numpy(raw).cuda()
    desc = cp.batch_desc(d.data_ptr(), 2, 65536, 16)
    lib = _abi.lib()
    for i in range(60):
        msg, ref = frames[i % 3]
        assert_same_detection(pipe.cloud_handler(msg), ref, f"single {i}")
        _abi.check(lib.cg_run_batch(pipe.handle, C.byref(desc), cp.CG_MODE_PIPELINE, None))
        r = _abi.cg_detect_result()
        _abi.check(lib.cg_batch_fetch(pipe.handle, i % 2, C.byref(r)))
        assert_same_detection(cp._detection(r), brefs[i % 2], f"batch {i}")


@pytest.mark.parametrize("frame", [0, 3])
def test_detector_matches_oracle(params, det, frame):
    raw = cp.synth_frames(1, first_frame=frame, rings=64, cols=1024)
    msg = cp.frame_cloud(raw[0])
    got = det.cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_DETECT)
    assert_same_detection(got, ref, f"detect f{frame}")


@pytest.mark.parametrize("frame", [0, 9])
def test_ground_removal_matches_oracle(params, ground, frame):
    raw = cp.synth_frames(1, first_frame=frame, rings=64, cols=1024)
    msg = cp.frame_cloud(raw[0])
    out = ground.cloud_handler(msg)
    ref, hdr = O.run(params, msg, O.MODE_GROUND)
    assert out.n_kept == int(hdr[1])
    g = out.data.view(np.float32).reshape(-1, 8)
    r = ref.view(np.float32).reshape(-1, 8)
    # declared fields x, y, z, intensity (+ data[3] = 1); PCL padding bytes are undefined
    cols = [0, 1, 2, 3, 4]
    assert np.array_equal(g[:, cols].view(np.uint32), r[:, cols].view(np.uint32))


def test_pcl32_layout_matches_xyzi16(params, pipe):
    raw16 = cp.synth_frames(1, first_frame=2, rings=64, cols=1024, point_step=16)
    raw32 = cp.synth_frames(1, first_frame=2, rings=64, cols=1024, point_step=32)
    a = pipe.cloud_handler(cp.frame_cloud(raw16[0], 16))
    b = pipe.cloud_handler(cp.frame_cloud(raw32[0], 32))
    ref, _ = O.run(params, cp.frame_cloud(raw32[0], 32), O.MODE_PIPELINE)
    assert_same_detection(a, ref, "xyzi16")
    assert_same_detection(b, ref, "pcl32")


def test_batch_engine_matches_oracle(params):
    import torch
    nf = 24
    raw = cp.synth_frames(nf, first_frame=100, rings=64, cols=1024)
    d = torch.from_numpy(raw).cuda()
    eng = cp.BatchEngine(params)
    eng.run(d.data_ptr(), nf, 65536, 16, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for f in range(nf):
        got = eng.fetch(f)
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE)
        assert_same_detection(got, ref, f"batch frame {f}")


@pytest.mark.parametrize("clutter,cpr,frame", [(20, 8, 0), (20, 8, 1), (60, 10, 0), (200, 10, 0)])
def test_dense_frames_match_oracle(params, pipe, clutter, cpr, frame):
    """Cluttered scenes: M > 512 (bitonic voxel sort), V > 384 (neighbour-grid clustering),
    C > 16 (PCL's introsort cluster order), M > 2048 (HBM-scratch backend)."""
    raw = cp.synth_frames(1, first_frame=frame, rings=64, cols=1024, clutter=clutter, cones_per_row=cpr)
    msg = cp.frame_cloud(raw[0])
    got = pipe.cloud_handler(msg)
    ref, hdr = O.run(params, msg, O.MODE_PIPELINE)
    assert_same_detection(got, ref, f"clutter {clutter} f{frame}")
    if int(hdr[2]) > 2048:
        assert got.flags & cp.CG_F_GLOBAL_SCRATCH


def test_dense_batch_mixed_paths(params):
    """One batch mixing LDS-path and HBM-scratch-path frames."""
    import torch
    raws = [cp.synth_frames(1, first_frame=f, rings=64, cols=1024, clutter=c, cones_per_row=8)[0]
            for f, c in ((0, 0), (1, 60), (2, 20), (3, 200), (4, 0))]
    raw = np.stack(raws)
    d = torch.from_numpy(raw).cuda()
    eng = cp.BatchEngine(params)
    eng.run(d.data_ptr(), raw.shape[0], 65536, 16, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for f in range(raw.shape[0]):
        ref, _ = O.run(params, cp.frame_cloud(raw[f]), O.MODE_PIPELINE)
        assert_same_detection(eng.fetch(f), ref, f"mixed batch frame {f}")


import kat_clouds as KC  # noqa: E402

_KATS = KC.all_kats()


@pytest.mark.parametrize("kat", _KATS, ids=[k[0] for k in _KATS])
@pytest.mark.parametrize("mode", ["pipeline", "detect", "ground"])
def test_kat_gpu_matches_oracle(kat, mode):
    """Known-answer edge clouds through the C-ABI single-frame calls vs the CPU restatement."""
    name, pts, over, _ = kat
    params = cp.load_params("simulation", over)
    msg = cp.PointCloud2.from_xyzi(pts)
    if mode == "ground":
        out = cp.GroundRemover(params).cloud_handler(msg)
        ref, hdr = O.run(params, msg, O.MODE_GROUND)
        assert out.n_kept == int(hdr[1]), name
        g = out.data.view(np.float32).reshape(-1, 8)
        r = ref.view(np.float32).reshape(-1, 8)
        assert np.array_equal(g[:, :5].view(np.uint32), r[:, :5].view(np.uint32)), name
        return
    eng = cp.ConePipeline(params) if mode == "pipeline" else cp.ConeDetector(params)
    got = eng.cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_PIPELINE if mode == "pipeline" else O.MODE_DETECT)
    assert_same_detection(got, ref, f"{name}/{mode}")


def test_detector_missing_intensity_quirk(params):
    """src/cone_detection.cpp:142-151: a detector input without an intensity field gets a
    fake FLOAT32 field at offset 0, so intensity reads x."""
    raw = cp.synth_frames(1, first_frame=3, rings=16, cols=1024)
    msg = cp.frame_cloud(raw[0])
    msg.fields = [f for f in msg.fields if f.name != "intensity"]
    det = cp.ConeDetector(params)
    got = det.cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_DETECT, intensity_offset=0)
    assert_same_detection(got, ref, "no-intensity detector")
    assert np.array_equal(got.voxels[:, 3].view(np.uint32), ref.voxels[:, 3].view(np.uint32))


def test_cpp_node_mirror_two_node_equals_fused():
    """The C++ mirror of the reference nodes (host/cones_nodes.hpp): GroundRemover ->
    groundless_cloud (PCL PointXYZI layout) -> ConeDetector equals the fused pipeline."""
    import subprocess
    from cones_perception_amd import build as B
    exe = B.build_host_demo()
    r = subprocess.run([exe, "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("two-node == fused") == 3
