"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py): the CPU
restatement must reproduce them bit for bit here and on the GPU box (same image), and the
GPU path must reproduce them too (gpu marker)."""
import glob
import json
import os

import numpy as np
import pytest

import cones_perception_amd as cp
import oracle_py as O
from helpers import same_bits

GOLD = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
              if os.path.basename(p) != "cones_csv.npz")   # the colour-classifier crops (test_colornet.py)
MODES = (("pipeline", O.MODE_PIPELINE), ("detect", O.MODE_DETECT), ("ground", O.MODE_GROUND))


def load(path):
    z = np.load(path, allow_pickle=False)
    over = json.loads(str(z["params"]))
    ps = int(z["point_step"])
    raw = z["input"]
    msg = cp.frame_cloud(raw, ps) if raw.size else cp.PointCloud2.from_xyzi(np.zeros((0, 4), np.float32))
    return z, cp.load_params("simulation", over), msg


def check(z, tag, hdr, det=None, ground=None):
    assert np.array_equal(hdr[:6], z[f"{tag}_hdr"][:6]), tag
    if ground is not None:
        g = ground.view(np.float32).reshape(-1, 8)[:, :5]
        r = z[f"{tag}_ground"].view(np.float32).reshape(-1, 8)[:, :5]
        assert np.array_equal(g.view(np.uint32), r.view(np.uint32)), tag
        return
    assert same_bits(det.voxels, z[f"{tag}_voxels"]), tag
    assert np.array_equal(det.labels, z[f"{tag}_labels"]), tag
    assert np.array_equal(det.cluster_offsets, z[f"{tag}_offsets"]), tag
    assert np.array_equal(det.cluster_indices, z[f"{tag}_indices"]), tag
    assert same_bits(det.centroids, z[f"{tag}_centroids"]), tag


def test_golden_present():
    assert len(GOLD) >= 12


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_oracle_reproduces_golden(path):
    z, params, msg = load(path)
    for tag, mode in MODES:
        out, hdr = O.run(params, msg, mode)
        if mode == O.MODE_GROUND:
            check(z, tag, hdr, ground=out)
        else:
            check(z, tag, hdr, det=out)


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_gpu_reproduces_golden(path):
    z, params, msg = load(path)
    got = cp.ConePipeline(params).cloud_handler(msg)
    check(z, "pipeline", np.array([got.n_points, got.n_kept, got.n_filtered, len(got.voxels),
                                   len(got.centroids), got.flags & 1], np.uint32), det=got)
    got = cp.ConeDetector(params).cloud_handler(msg)
    check(z, "detect", np.array([got.n_points, got.n_kept, got.n_filtered, len(got.voxels),
                                 len(got.centroids), got.flags & 1], np.uint32), det=got)
    g = cp.GroundRemover(params).cloud_handler(msg)
    n = msg.width * msg.height
    check(z, "ground", np.array([n, g.n_kept, 0, 0, 0, 0], np.uint32), ground=g.data)
