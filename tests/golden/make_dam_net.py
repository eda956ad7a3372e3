"""Writes tests/golden/dam_net_weights.npy: the reference's dam_net colour classifier weights
(models/dam_net/dam_net.tflite), packed as cg_colornet_set takes them, read by
cones_perception_amd.colornet.read_tflite (flatbuffer data only; nothing is executed).

Pins the .tflite reading against the reference's other copy of the same model, its SavedModel
checkpoint (models/dam_net/variables/variables.data-00000-of-00001, raw little-endian float32
tensors): the conv and dense kernels, transposed to TF's HWIO / IO layouts, and the biases are
found there byte for byte, and the .tflite graph's MUL / ADD constants equal the checkpoint's
batch norm folded as gamma / sqrt(var + 1e-3) and beta - mean * scale to float32 rounding.

Run in the build container (needs /root/reference): python tests/golden/make_dam_net.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from cones_perception_amd.colornet import read_tflite  # noqa: E402

REF = "/root/reference/models/dam_net"


def unpack(w):
    shapes = [(16, 3, 3, 1), (16,), (32, 3, 3, 16), (32,), (32,), (32,), (3, 64), (3,)]
    out, k = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(w[k:k + n].reshape(s))
        k += n
    return out


def pin(w):
    data = open(os.path.join(REF, "variables", "variables.data-00000-of-00001"), "rb").read()
    w1, b1, w2, b2, bnm, bna, wd, bd = unpack(w)
    found = {}
    for name, a in [("conv2d/kernel", w1.transpose(1, 2, 3, 0)), ("conv2d/bias", b1),
                    ("conv2d_1/kernel", w2.transpose(1, 2, 3, 0)), ("conv2d_1/bias", b2),
                    ("dense/kernel", wd.T), ("dense/bias", bd)]:
        at = data.find(np.ascontiguousarray(a, "<f4").tobytes())
        assert at >= 0, f"{name} not in the checkpoint"
        found[name] = at
    # the four batch-norm vectors sit between conv2d_1/bias and dense/kernel
    lo = found["conv2d_1/bias"] + 128
    g, b, m, v = np.frombuffer(data[lo:lo + 512], "<f4").reshape(4, 32).astype(np.float64)
    scale = g / np.sqrt(v + 1e-3)
    assert np.allclose(scale, bnm, rtol=0, atol=1e-6), "batch-norm scale"
    assert np.allclose(b - m * scale, bna, rtol=0, atol=1e-6), "batch-norm offset"
    return found


if __name__ == "__main__":
    w = read_tflite(os.path.join(REF, "dam_net.tflite"))
    print("pinned against the SavedModel checkpoint at", pin(w))
    np.save(os.path.join(HERE, "dam_net_weights.npy"), w)
    print("wrote", os.path.join(HERE, "dam_net_weights.npy"), w.shape)
