"""Adversarial frames for pass 1's certified classification (sector rays, approximate atan2,
angle-filter classes): points packed around every 22-degree sector edge
(src/ground_removal.cpp:61-64) and around the +-angle_threshold edges
(src/cone_detection.cpp:200-201), laid out so that a wrong sector or angle class for any of
them changes the frame's results.

- Probes: per sector edge, points at angle edge +- delta with |delta| spread over 1e-8..1e-2
  rad. The probes of one |delta| band (the frame's `band`) are the lowest points of their
  sector, so each sector's minimum - and so its ground threshold min + 0.1 - is set by a probe
  of that band: a probe counted in the wrong sector moves two thresholds.
- Ladder: per sector, points at mid-wedge angles whose z climb through the threshold window in
  0.1 mm steps, so any threshold shift changes the kept count K.
- Filter probes: points around +-angle_threshold, above the ground, inside the distance band:
  a wrong angle class changes the detector input (M) and the voxels.
- Filler: ground at random angles.

`order` "angle" sorts the points by azimuth (a lane's consecutive points, 512 apart, mostly
share a sector, as on a spinning sensor: the ray fast path); "shuffled" is random order (the
fallback path at nearly every point).
"""
import numpy as np

SEC = np.float64(np.float32(22 * np.pi / 180))       # the reference's float sector width
BANDS = [(1e-8, 1e-6), (1e-6, 1e-5), (1e-5, 1.9e-5), (1.9e-5, 3e-5), (3e-5, 1e-4), (1e-4, 1e-2)]


def sector_edge_frame(band, order="angle", n=65536, seed=0, theta_deg=160.0):
    rng = np.random.default_rng(seed * 131 + band)
    lo_d, hi_d = BANDS[band]
    pts = []
    # probes around each sector edge (edge 0 = the 0 / 2 pi wrap between bins 16 and 0)
    edges = np.arange(17, dtype=np.float64) * SEC
    n_probe = 256
    for e in edges:
        mag = np.exp(rng.uniform(np.log(1e-8), np.log(1e-2), n_probe))
        inb = rng.random(n_probe) < 0.5
        mag[inb] = np.exp(rng.uniform(np.log(lo_d), np.log(hi_d), inb.sum()))
        a = e + mag * np.where(rng.random(n_probe) < 0.5, -1.0, 1.0)
        r = rng.uniform(2.0, 9.0, n_probe)
        z = np.where(inb, rng.uniform(-0.95, -0.90, n_probe), rng.uniform(-0.80, -0.70, n_probe))
        pts.append(np.stack([r * np.cos(a), r * np.sin(a), z, np.full(n_probe, 1.0)], 1))
    # ladders: z from -0.90 to -0.70 at mid-wedge angles of every sector (bin 16 is 8 deg wide),
    # beyond distance_treshold_max (they count in K, not in the detector input)
    n_lad = 1800
    for s in range(17):
        w0, w1 = s * SEC, min((s + 1) * SEC, 2 * np.pi)
        a = rng.uniform(w0 + 0.2 * (w1 - w0), w0 + 0.8 * (w1 - w0), n_lad)
        r = rng.uniform(10.5, 20.0, n_lad)
        z = np.linspace(-0.90, -0.70, n_lad) + rng.uniform(-2e-5, 2e-5, n_lad)
        pts.append(np.stack([r * np.cos(a), r * np.sin(a), z, np.full(n_lad, 2.0)], 1))
    # angle-filter probes around +-theta, above the ground, 2-9 m out
    th = np.deg2rad(theta_deg)
    n_f = 512
    for sgn in (1.0, -1.0):
        mag = np.exp(rng.uniform(np.log(1e-8), np.log(1e-2), n_f))
        a = sgn * th + mag * np.where(rng.random(n_f) < 0.5, -1.0, 1.0)
        r = rng.uniform(2.0, 9.0, n_f)
        z = rng.uniform(-0.2, 0.3, n_f)
        pts.append(np.stack([r * np.cos(a), r * np.sin(a), z, np.full(n_f, 3.0)], 1))
    p = np.concatenate(pts)
    # filler: ground below every threshold, above every sector minimum, at random angles
    k = n - p.shape[0]
    assert k >= 0, "frame too small for the probes"
    a = rng.uniform(0, 2 * np.pi, k)
    r = rng.uniform(1.5, 20.0, k)
    fill = np.stack([r * np.cos(a), r * np.sin(a), rng.uniform(-0.89, -0.86, k), np.full(k, 4.0)], 1)
    p = np.concatenate([p, fill]).astype(np.float32)
    if order == "angle":
        az = np.arctan2(p[:, 1].astype(np.float64), p[:, 0].astype(np.float64)) % (2 * np.pi)
        p = p[np.argsort(az, kind="stable")]
    else:
        p = p[rng.permutation(p.shape[0])]
    return np.ascontiguousarray(p)
