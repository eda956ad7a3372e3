"""Hand-built known-answer clouds for the edge semantics of SURVEY.md §8.1.

Each builder returns (name, xyzi points (N, 4) float32, params overrides, expectation dict).
Expectations are derived by hand from the reference's expressions (cited per case); the
tests check them on the CPU restatement (oracle), the numpy restatement, and the GPU.
"""
import numpy as np

F32 = np.float32


def _cone(cx, cy, n_side=6, z0=-0.5, h=0.3, r=0.1):
    """A compact blob of points (one cluster) around (cx, cy)."""
    pts = []
    for a in range(n_side):
        for b in range(3):
            ang = 2 * np.pi * a / n_side
            rr = r * (1 - b / 3)
            pts.append([cx + rr * np.cos(ang), cy + rr * np.sin(ang), z0 + h * b / 3, 10.0])
    return np.array(pts, F32)


def ground_grid(r0=1.2, r1=9.0, nr=24, nth=90, z=-0.5):
    pts = []
    for i in range(nr):
        rr = r0 + (r1 - r0) * i / (nr - 1)
        for j in range(nth):
            th = -np.pi + 2 * np.pi * (j + 0.5) / nth
            pts.append([rr * np.cos(th), rr * np.sin(th), z, 5.0])
    return np.array(pts, F32)


def kat_ground_threshold():
    """G4: keep iff !((double)z < (double)low + 0.1). With low = -0.5f the threshold is
    -0.4 (double); float(-0.4) = -0.4000000059604645 is below it (removed), its float
    neighbour toward zero (-0.39999998) is kept (src/ground_removal.cpp:75)."""
    g = ground_grid()
    # both probes in the sector of angle ~ 10 deg (sector 0), far from ground points' z
    a = np.deg2rad(10.0)
    probes = np.array([[3 * np.cos(a), 3 * np.sin(a), F32(-0.4), 1.0],
                       [3.1 * np.cos(a), 3.1 * np.sin(a), np.nextafter(F32(-0.4), F32(0)), 2.0]], F32)
    pts = np.concatenate([g, probes])
    return "ground_threshold", pts, {}, {"ground_kept_probe_intensities": [2.0]}


def kat_sector16():
    """G1/G3: sectors are 22 deg wide; angles in [352, 360) deg form bin 16, its own bin here.
    A very low point in bin 16 must not lower the threshold of bins 15 or 0."""
    g = ground_grid(z=-0.5)
    a16 = np.deg2rad(355.0)
    a0 = np.deg2rad(3.0)
    deep = np.array([[4 * np.cos(a16), 4 * np.sin(a16), -3.0, 7.0]], F32)          # bin 16 min
    obj0 = np.array([[4 * np.cos(a0), 4 * np.sin(a0), -0.35, 8.0]], F32)           # bin 0 object
    obj16 = np.array([[4.2 * np.cos(a16), 4.2 * np.sin(a16), -0.45, 9.0]], F32)    # bin 16: kept
    pts = np.concatenate([g, deep, obj0, obj16])
    return "sector16", pts, {}, {"kept_intensities_include": [8.0, 9.0]}


def kat_tolerance():
    """E1: edge iff fl((dx^2 + dy^2) + dz^2) < r2f (strict). r = float(sqrt(0.325f^2 +
    0.228f^2)) = 0.39699998f, r2f = float(r*r) = 0.15760899f. Two pairs along x at
    separations whose float squares straddle r2f."""
    r = F32(0.39699998)
    r2 = F32(np.float64(r) * np.float64(r))
    base = np.array([[3.0, 0.0, -0.3, 1.0]], F32)
    # x2 - 4 is exact (Sterbenz), so the float predicate sees dx = x2 - 4 exactly
    x0 = F32(4.0)
    x2 = F32(4.0 + 0.397)
    while F32(F32(x2 - x0) * F32(x2 - x0)) >= r2:
        x2 = np.nextafter(x2, F32(0))
    x_lo = x2                                  # largest x2 whose pair is connected
    x_hi = np.nextafter(x2, F32(10))           # smallest x2 whose pair is not
    assert F32(F32(x_hi - x0) ** 2) >= r2 > F32(F32(x_lo - x0) ** 2)
    pa = np.array([[x0, 2.0, -0.3, 1.0], [x_lo, 2.0, -0.3, 1.0]], F32)
    pb = np.array([[x0, -2.0, -0.3, 1.0], [x_hi, -2.0, -0.3, 1.0]], F32)
    pts = np.concatenate([base, pa, pb])
    return "tolerance", pts, {"min_cluster_size": 1}, {"sizes": [2, 1, 1, 1]}


def kat_cluster_sizes():
    """E3: keep clusters with min <= size <= max (unsigned compare); sizes 1, 2, 3, 4 with
    min = 2, max = 3 keep exactly the clusters of 2 and 3 voxels."""
    pts = []
    for k, n in enumerate([1, 2, 3, 4]):
        cx, cy = 3.0 + 1.5 * k, 0.5
        for j in range(n):
            pts.append([cx + 0.05 * j, cy, -0.3, 1.0])   # one point per 4 cm voxel
    return "cluster_sizes", np.array(pts, F32), {"min_cluster_size": 2, "max_cluster_size": 3}, \
        {"sizes": [3, 2]}


def kat_many_equal_clusters():
    """E4: more than 16 clusters of equal size: PCL's order is std::sort's (introsort)
    permutation of the reversed discovery list, not (size desc, seed asc)."""
    pts = []
    rng = np.random.default_rng(5)
    k = 0
    for ix in range(6):
        for iy in range(6):
            cx, cy = 1.5 + 1.0 * ix, -3.0 + 1.0 * iy
            n = 2 if (k % 3) else 3
            for j in range(n):
                pts.append([cx + 0.05 * j, cy + rng.uniform(-0.004, 0.004), -0.3, 1.0])
            k += 1
    return "many_equal_clusters", np.array(pts, F32), {"min_cluster_size": 2}, {"n_clusters_min": 17}


def kat_voxel_passthrough():
    """V2: if dx*dy*dz > INT32_MAX the VoxelGrid returns its input unchanged."""
    pts = np.array([[1.5, 0.0, -0.3, 1.0], [150.0, 0.3, -0.3, 2.0], [2.0, 150.0, 9.0, 3.0],
                    [1.52, 0.01, -0.3, 4.0]], F32)
    over = {"distance_treshold_max": 1000.0, "angle_threshold": 179.0, "level_threshold": -50.0}
    return "voxel_passthrough", pts, over, {"passthrough": True}


def kat_zero_pad_survives():
    """G5 + D1: the groundless cloud ends with N-K PointXYZI() (0,0,0); they survive the
    filter iff 0 >= dmin etc. With distance_treshold_min = 0 they do (d = 0 is not < 0),
    form one voxel at the origin, and a cluster if min_cluster_size <= 1."""
    g = ground_grid(nr=6, nth=24)
    pts = np.concatenate([g, _cone(3.0, 0.5)])
    over = {"distance_treshold_min": 0.0, "min_cluster_size": 1}
    return "zero_pad_survives", pts, over, {"origin_voxel": True}


def kat_empty():
    return "empty", np.zeros((0, 4), F32), {}, {"n_clusters": 0}


def kat_all_filtered():
    pts = np.array([[0.1, 0.1, 0.0, 1.0], [50.0, 0.0, 0.0, 1.0], [-5.0, 0.01, 0.0, 1.0]], F32)
    return "all_filtered", pts, {}, {"n_filtered": 0}


def kat_nonfinite():
    """NaN/inf points: NaN survives the reference's filter comparisons (all false), VoxelGrid
    drops non-finite points (getMinMax3D / idx loop skip them)."""
    g = ground_grid(nr=4, nth=24)
    c = _cone(4.0, 1.0)
    bad = np.array([[np.nan, 1.0, -0.3, 1.0], [3.0, 0.5, np.nan, 1.0], [np.inf, 0.0, -0.3, 1.0]], F32)
    return "nonfinite", np.concatenate([g, c, bad]), {}, {}


def all_kats():
    return [kat_ground_threshold(), kat_sector16(), kat_tolerance(), kat_cluster_sizes(),
            kat_many_equal_clusters(), kat_voxel_passthrough(), kat_zero_pad_survives(), kat_empty(),
            kat_all_filtered(), kat_nonfinite()]
