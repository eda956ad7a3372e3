"""GPU parity of the device-sized PCL-order partition (cg_large.hip lg_pq_flow) on index_vectors
built to stress it: keys already sorted, reversed, all equal, a few values interleaved, and
random keys with heavy duplication. Each cloud holds 100,000 points inside the position filter,
so the detector's frame takes the device-sized path with more tiles in range 0 (196) than the
launch has workgroups (192): range 0's early tiles defer their swaps. Voxel sums depend on
std::sort's exact permutation of equal keys (float sums in that order), so voxel bits match
the oracle's ORDER_PCL only if the partition reproduces libstdc++'s introsort exactly
(src/cone_detection.cpp:240-249, PCL 1.10 VoxelGrid). The tile-level protocol of these
shapes is modelled on the CPU in tests/test_pq_flow_model.py."""
import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import assert_same_detection

pytestmark = pytest.mark.gpu

N = 100_000
LEAF = 0.04   # the simulation profile's voxel leaf


def _grid_points(order):
    """N points on a 0.04 m grid inside the filter (1 m <= range <= 10 m, |angle| < 160 deg),
    two points per voxel (jittered inside it), listed so that their voxel keys run in `order`."""
    rng = np.random.default_rng(7)
    nx, ny, nz = 125, 50, 8          # 50,000 voxels: keys i0 + i1 nx + i2 nx ny
    i = np.arange(N) // 2
    i0, i1, i2 = i % nx, (i // nx) % ny, i // (nx * ny)
    x = 3.0 + (i0 + 0.25 + 0.5 * rng.random(N)) * LEAF
    y = -1.0 + (i1 + 0.25 + 0.5 * rng.random(N)) * LEAF
    z = -0.5 + (i2 + 0.25 + 0.5 * rng.random(N)) * LEAF
    pts = np.stack([x, y, z, np.ones(N)], axis=1).astype(np.float32)
    if order == "descending":
        pts = pts[::-1].copy()
    elif order == "random_dup":
        pts = pts[rng.permutation(N)]
    return pts


def _one_voxel():
    rng = np.random.default_rng(11)
    x = 3.0 + (0.1 + 0.8 * rng.random(N)) * LEAF
    y = 0.52 + (0.1 + 0.8 * rng.random(N)) * LEAF
    z = 0.0 + (0.1 + 0.8 * rng.random(N)) * LEAF
    return np.stack([x, y, z, rng.random(N) * 100.0], axis=1).astype(np.float32)


def _three_voxels():
    """Keys cycling over three voxels: long runs of ties, and every cut uneven."""
    rng = np.random.default_rng(13)
    v = np.arange(N) % 3
    x = 3.0 + (v * 5 + 0.1 + 0.8 * rng.random(N)) * LEAF
    y = 0.52 + (0.1 + 0.8 * rng.random(N)) * LEAF
    z = 0.0 + (0.1 + 0.8 * rng.random(N)) * LEAF
    return np.stack([x, y, z, rng.random(N) * 100.0], axis=1).astype(np.float32)


CASES = {
    "ascending": lambda: _grid_points("ascending"),
    "descending": lambda: _grid_points("descending"),
    "random_dup": lambda: _grid_points("random_dup"),
    "one_voxel": _one_voxel,
    "three_voxels": _three_voxels,
}


@pytest.mark.parametrize("case", list(CASES))
def test_flow_partition_edge_clouds(case):
    params = cp.load_params("simulation")
    pts = CASES[case]()
    msg = cp.PointCloud2.from_xyzi(pts)
    got = cp.ConeDetector(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_DETECT)
    assert ref.n_filtered == N, ref.n_filtered   # every point reaches the voxel stage
    assert_same_detection(got, ref, f"flow edge {case}")


@pytest.mark.parametrize("n_keep", [2048, 2049, 2561, 4097, 70_001])
def test_flow_index_vector_lengths(n_keep):
    """A 70,001-point cloud (the device-sized path) of which n_keep points reach the voxel stage
    (the rest lie past distance_treshold_max): index_vectors at and just past one leaf (2,048:
    no partition at all; 2,049: the smallest range the launch cuts), a few tiles, and nearly the
    whole cloud. Random voxel keys with duplicates."""
    params = cp.load_params("simulation")
    rng = np.random.default_rng(n_keep)
    n_all = 70_001
    pts = np.zeros((n_all, 4), np.float32)
    k = rng.integers(0, max(2, n_keep // 3), n_all)      # ~3 points per voxel
    pts[:, 0] = 3.0 + ((k % 97) + 0.5) * LEAF
    pts[:, 1] = -1.0 + (((k // 97) % 41) + 0.5) * LEAF
    pts[:, 2] = -0.5 + ((k // (97 * 41)) + 0.5) * LEAF
    pts[:, 3] = rng.random(n_all) * 100.0
    far = rng.permutation(n_all)[: n_all - n_keep]
    pts[far, 0] = 20.0                                    # past the 10 m filter
    msg = cp.PointCloud2.from_xyzi(pts)
    got = cp.ConeDetector(params).cloud_handler(msg)
    ref, _ = O.run(params, msg, O.MODE_DETECT)
    assert ref.n_filtered == n_keep, ref.n_filtered
    assert_same_detection(got, ref, f"index_vector {n_keep}")
