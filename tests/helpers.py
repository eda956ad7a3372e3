"""Shared comparison helpers for parity tests."""
import numpy as np


def same_bits(a, b):
    """Bit-identical float arrays, except that any NaN equals any NaN (x86 and gfx950 differ
    in the sign of a default NaN, e.g. the 0/0 centroid of an origin-only cluster)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    if a.shape != b.shape:
        return False
    nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(nan | (a.view(np.uint32) == b.view(np.uint32))))


def assert_same_detection(got, ref, ctx=""):
    """Bit-exact comparison of two Detection results (GPU vs CPU restatement)."""
    assert got.n_points == ref.n_points, ctx
    assert got.n_kept == ref.n_kept, f"{ctx} K {got.n_kept} != {ref.n_kept}"
    assert got.n_filtered == ref.n_filtered, f"{ctx} M {got.n_filtered} != {ref.n_filtered}"
    assert got.voxels.shape == ref.voxels.shape, f"{ctx} V {got.voxels.shape} != {ref.voxels.shape}"
    assert same_bits(got.voxels, ref.voxels), f"{ctx} voxel bits differ"
    assert np.array_equal(got.cluster_offsets, ref.cluster_offsets), f"{ctx} cluster sizes/order differ"
    assert np.array_equal(got.cluster_indices, ref.cluster_indices), f"{ctx} cluster index sets differ"
    assert np.array_equal(got.labels, ref.labels), f"{ctx} labels differ"
    assert same_bits(got.centroids, ref.centroids), \
        f"{ctx} centroid bits differ: max abs {np.nanmax(np.abs(got.centroids - ref.centroids)) if got.centroids.size else 0}"
    assert (got.flags & 1) == (ref.flags & 1), f"{ctx} passthrough flag"


def assert_same_cluster_sets(got, ref, ctx="", tol=1e-5):
    """The north star's bar (BASELINE.json): cluster index sets identical to the reference's
    (same voxel count, sizes, order and members) and centroids within `tol` metres. Used where
    the voxel sums legitimately run in another order than PCL's (the halo form's slabs)."""
    assert got.n_points == ref.n_points and got.n_kept == ref.n_kept and got.n_filtered == ref.n_filtered, ctx
    assert got.voxels.shape == ref.voxels.shape, f"{ctx} V {got.voxels.shape} != {ref.voxels.shape}"
    assert np.array_equal(got.cluster_offsets, ref.cluster_offsets), f"{ctx} cluster sizes/order differ"
    assert np.array_equal(got.cluster_indices, ref.cluster_indices), f"{ctx} cluster index sets differ"
    assert got.centroids.shape == ref.centroids.shape, ctx
    if got.centroids.size:
        d = np.abs(got.centroids.astype(np.float64) - ref.centroids.astype(np.float64))
        fin = np.isfinite(d)
        assert np.array_equal(np.isnan(got.centroids), np.isnan(ref.centroids)), ctx
        assert (not fin.any()) or float(d[fin].max()) <= tol, f"{ctx} centroid error {float(d[fin].max())} > {tol}"
