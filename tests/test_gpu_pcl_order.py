"""GPU parity against PCL's own voxel order. In its default mode (CG_VOXEL_ORDER_PCL) the
device reproduces VoxelGrid's std::sort(index_vector) permutation (cg_pcl.h), so voxel sums
run in PCL's order and every output is bit-identical to the oracle's ORDER_PCL mode; in
CG_VOXEL_ORDER_POINT mode it is bit-identical to ORDER_STABLE and flags the results, and its
cluster index sets equal PCL's with centroids within the north star's 1e-5 m.

Inputs: C1/C2 frames, cluttered frames (M > 512, V > 256, C > 16, the HBM-scratch backend),
the known-answer clouds, C3 as configured (256 x 64k frames on three batch engines, three
HIP streams in flight), and the large path (a 128-ring detector frame with 64k survivors, the
1M-point C5 frame). Each case also counts the frames whose voxel bits differ between PCL's
order and ascending point order, i.e. the cases this parity distinguishes.
"""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import assert_same_detection, same_bits
from kat_clouds import all_kats

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def params():
    return cp.load_params("simulation")


def _check(got, params, msg, mode, ctx, stats=None):
    ref, _ = O.run(params, msg, mode, order=O.ORDER_PCL)
    assert_same_detection(got, ref, ctx)
    if stats is not None:
        st, _ = O.run(params, msg, mode, order=O.ORDER_STABLE)
        stats["frames"] += 1
        stats["order_matters"] += int(not same_bits(st.voxels, ref.voxels))


@pytest.mark.parametrize("rings,clutter,cpr,mode", [(16, 0, 5, "pipeline"), (64, 0, 5, "pipeline"),
                                                    (64, 0, 5, "detect"), (64, 20, 8, "pipeline"),
                                                    (64, 60, 10, "pipeline"), (64, 200, 10, "pipeline"),
                                                    (64, 60, 10, "detect")])
def test_frames_match_pcl_order(params, rings, clutter, cpr, mode):
    stats = {"frames": 0, "order_matters": 0}
    eng = cp.ConePipeline(params) if mode == "pipeline" else cp.ConeDetector(params)
    om = O.MODE_PIPELINE if mode == "pipeline" else O.MODE_DETECT
    for f in range(4):
        raw = cp.synth_frames(1, first_frame=30 + f, rings=rings, cols=1024, clutter=clutter, cones_per_row=cpr)
        msg = cp.frame_cloud(raw[0])
        _check(eng.cloud_handler(msg), params, msg, om, f"{rings} rings clutter {clutter} f{f} {mode}", stats)
    print(f"PCL-order frames {stats['frames']}, voxel bits order-dependent in {stats['order_matters']}")
    if clutter == 0 and rings == 64:
        assert stats["order_matters"] > 0   # the comparison can tell the two orders apart


_KATS = all_kats()


@pytest.mark.parametrize("kat", _KATS, ids=[k[0] for k in _KATS])
def test_kats_match_pcl_order(kat):
    name, pts, over, _ = kat
    params = cp.load_params("simulation", over)
    msg = cp.PointCloud2.from_xyzi(pts)
    _check(cp.ConePipeline(params).cloud_handler(msg), params, msg, O.MODE_PIPELINE, name)
    _check(cp.ConeDetector(params).cloud_handler(msg), params, msg, O.MODE_DETECT, name)


def test_c3_three_streams_match_pcl_order(params):
    """C3 as the bench runs it: 256 frames x 65,536 points per batch, three batch engines on
    three HIP streams, launches in flight together; every frame of every engine's batch is
    compared with the oracle (PCL order), bit for bit."""
    import torch
    F, S = 256, 3
    dev = torch.device("cuda", 0)
    raws = [cp.synth_frames(F, first_frame=1000 + s * F, rings=64, cols=1024, threads=16) for s in range(S)]
    d = [torch.from_numpy(r).to(dev) for r in raws]
    engines = [cp.BatchEngine(params) for _ in range(S)]
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    torch.cuda.synchronize(dev)
    for step in range(2 * S):   # two launches per engine, three streams overlapping
        s = step % S
        engines[s].run(d[s].data_ptr(), F, 65536, 16, stream=streams[s].cuda_stream)
    torch.cuda.synchronize(dev)
    stats = {"frames": 0, "order_matters": 0}
    for s in range(S):
        for f in range(F):
            _check(engines[s].fetch(f), params, cp.frame_cloud(raws[s][f]), O.MODE_PIPELINE,
                   f"engine {s} frame {f}", stats if f < 64 else None)
    print(f"C3 3-stream: {S * F} frames bit-exact vs PCL order; order-dependent voxel bits in "
          f"{stats['order_matters']} of {stats['frames']} sampled")


@pytest.mark.parametrize("rings,cols,clutter,cpr,mode", [(64, 1024, 0, 5, "pipeline"), (64, 1024, 60, 10, "pipeline"),
                                                         (128, 1024, 0, 5, "detect"), (128, 8192, 60, 12, "pipeline")])
def test_point_order_mode(params, rings, cols, clutter, cpr, mode):
    """CG_VOXEL_ORDER_POINT: bit-exact against ORDER_STABLE, flagged, and against PCL's order
    identical cluster index sets with centroids within 1e-5 m (the north star's bar). The
    128 x 8192 frame is C5's 1M-point shape."""
    import numpy as np
    from helpers import same_bits
    eng = (cp.ConePipeline if mode == "pipeline" else cp.ConeDetector)(params).set_voxel_order(cp.CG_VOXEL_ORDER_POINT)
    om = O.MODE_PIPELINE if mode == "pipeline" else O.MODE_DETECT
    raw = cp.synth_frames(1, first_frame=2, rings=rings, cols=cols, clutter=clutter, cones_per_row=cpr)
    msg = cp.frame_cloud(raw[0])
    got = eng.cloud_handler(msg)
    st, _ = O.run(params, msg, om, order=O.ORDER_STABLE)
    assert_same_detection(got, st, f"point order {rings}x{cols}")
    assert got.flags & cp.CG_F_VOXEL_POINT_ORDER
    pcl, _ = O.run(params, msg, om, order=O.ORDER_PCL)
    assert np.array_equal(got.cluster_offsets, pcl.cluster_offsets)
    assert np.array_equal(got.cluster_indices, pcl.cluster_indices)
    if got.centroids.size:
        assert float(np.nanmax(np.abs(got.centroids.astype(np.float64) - pcl.centroids))) <= 1e-5
    # and the default mode on the same frame: PCL's bits
    got2 = (cp.ConePipeline if mode == "pipeline" else cp.ConeDetector)(params).cloud_handler(msg)
    assert_same_detection(got2, pcl, f"pcl order {rings}x{cols}")
    assert not got2.flags & cp.CG_F_VOXEL_POINT_ORDER
    print(f"{rings}x{cols} {mode}: voxel bits differ between the orders: {not same_bits(st.voxels, pcl.voxels)}")
