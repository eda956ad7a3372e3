"""Shared comparison helpers for parity tests."""
import numpy as np


def assert_same_detection(got, ref, ctx=""):
    """Bit-exact comparison of two Detection results (GPU vs CPU restatement)."""
    assert got.n_points == ref.n_points, ctx
    assert got.n_kept == ref.n_kept, f"{ctx} K {got.n_kept} != {ref.n_kept}"
    assert got.n_filtered == ref.n_filtered, f"{ctx} M {got.n_filtered} != {ref.n_filtered}"
    assert got.voxels.shape == ref.voxels.shape, f"{ctx} V {got.voxels.shape} != {ref.voxels.shape}"
    assert np.array_equal(got.voxels.view(np.uint32), ref.voxels.view(np.uint32)), f"{ctx} voxel bits differ"
    assert np.array_equal(got.cluster_offsets, ref.cluster_offsets), f"{ctx} cluster sizes/order differ"
    assert np.array_equal(got.cluster_indices, ref.cluster_indices), f"{ctx} cluster index sets differ"
    assert np.array_equal(got.labels, ref.labels), f"{ctx} labels differ"
    assert np.array_equal(got.centroids.view(np.uint32), ref.centroids.view(np.uint32)), \
        f"{ctx} centroid bits differ: max abs {np.abs(got.centroids - ref.centroids).max() if got.centroids.size else 0}"
    assert (got.flags & 1) == (ref.flags & 1), f"{ctx} passthrough flag"
