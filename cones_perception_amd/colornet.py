"""Colour classifier service on the GPU.

Mirrors ColorClassifier of the reference (scripts/color_classifier_server.py:40-156): the
ROS service `color_classifier` receives one point cloud per cone and answers one colour per
non-empty cloud (1 yellow, 2 blue, 3 orange, 0 unknown). The image construction (to_image)
and the dam_net CNN run in one HIP kernel (csrc/cg_colornet.hip) through the C-ABI
(cg_colornet_set, cg_classify_colors).

The model is the reference's TFLite file (its `~model_path` param). `read_tflite` reads the
graph's constants from the flatbuffer as data (no TensorFlow, nothing executed from the file)
and checks that the graph is the dam_net topology the kernel implements.
"""
import ctypes as C
import struct

import numpy as np

from . import _abi
from ._abi import check, lib

WEIGHTS = 5059
SKIPPED, INDEX_ERROR, RANGE_ERROR = -1, -2, -3
COLOR_NAMES = [None, "yellow", "blue", "orange"]   # color_classifier_server.py:76

# TFLite builtin operator codes and enums (tensorflow/lite/schema/schema.fbs)
_ADD, _CONV_2D, _FULLY_CONNECTED, _MAX_POOL_2D, _MUL, _RESHAPE, _SOFTMAX = 0, 3, 9, 17, 18, 22, 25
_VALID, _RELU, _NONE = 1, 1, 0


class _Flat:
    """Minimal flatbuffer table reader (little-endian, the TFLite schema's field numbers)."""

    def __init__(self, b):
        self.b = b

    def u32(self, p):
        return struct.unpack_from("<I", self.b, p)[0]

    def i32(self, p):
        return struct.unpack_from("<i", self.b, p)[0]

    def field(self, t, i):
        vt = t - self.i32(t)
        if 4 + 2 * i >= struct.unpack_from("<H", self.b, vt)[0]:
            return None
        o = struct.unpack_from("<H", self.b, vt + 4 + 2 * i)[0]
        return t + o if o else None

    def ref(self, p):
        return p + self.u32(p)

    def table(self, t, i):
        f = self.field(t, i)
        return None if f is None else self.ref(f)

    def vec(self, t, i):
        f = self.field(t, i)
        if f is None:
            return []
        v = self.ref(f)
        return [v + 4 + 4 * k for k in range(self.u32(v))]

    def ints(self, t, i):
        return [self.i32(p) for p in self.vec(t, i)]

    def scalar(self, t, i, fmt, default):
        f = self.field(t, i)
        return default if f is None else struct.unpack_from("<" + fmt, self.b, f)[0]

    def bytes_(self, t, i):
        f = self.field(t, i)
        if f is None:
            return b""
        v = self.ref(f)
        return self.b[v + 4: v + 4 + self.u32(v)]


def read_tflite(path):
    """The packed float32 weights (include/cones_gpu.h CG_COLORNET_WEIGHTS order) of a dam_net
    .tflite file. Raises ValueError if the graph is not dam_net's topology."""
    with open(path, "rb") as fh:
        b = fh.read()
    if b[4:8] != b"TFL3":
        raise ValueError(f"{path}: not a TFLite flatbuffer")
    F = _Flat(b)
    root = F.u32(0)
    codes = []
    for p in F.vec(root, 1):                           # Model.operator_codes
        oc = F.ref(p)
        codes.append(max(F.scalar(oc, 0, "b", 0), F.scalar(oc, 3, "i", 0)))
    subgraphs = F.vec(root, 2)
    if len(subgraphs) != 1:
        raise ValueError("expected one subgraph")
    sg = F.ref(subgraphs[0])
    tensors = [F.ref(p) for p in F.vec(sg, 0)]
    buffers = [F.ref(p) for p in F.vec(root, 4)]

    def const(ti, shape):
        t = tensors[ti]
        if F.scalar(t, 1, "b", 0) != 0:                # TensorType FLOAT32
            raise ValueError(f"tensor {ti}: not float32")
        if F.ints(t, 0) != list(shape):
            raise ValueError(f"tensor {ti}: shape {F.ints(t, 0)} != {list(shape)}")
        data = F.bytes_(buffers[F.scalar(t, 2, "I", 0)], 0)
        a = np.frombuffer(data, "<f4")
        if a.size != int(np.prod(shape)):
            raise ValueError(f"tensor {ti}: {a.size} values for shape {shape}")
        return a.astype(np.float32)

    ops = []
    for p in F.vec(sg, 3):
        o = F.ref(p)
        ops.append((codes[F.scalar(o, 0, "I", 0)], F.ints(o, 1), F.ints(o, 2), F.table(o, 4)))
    want = [_CONV_2D, _MAX_POOL_2D, _CONV_2D, _MAX_POOL_2D, _MUL, _ADD, _RESHAPE, _FULLY_CONNECTED, _SOFTMAX]
    if [op[0] for op in ops] != want:
        raise ValueError(f"operator sequence {[op[0] for op in ops]} is not dam_net's {want}")
    for k in (0, 2):                                   # Conv2DOptions: VALID, stride 1, ReLU, no dilation
        opt = ops[k][3]
        if (F.scalar(opt, 0, "b", 0), F.scalar(opt, 1, "i", 0), F.scalar(opt, 2, "i", 0),
                F.scalar(opt, 3, "b", 0), F.scalar(opt, 4, "i", 1), F.scalar(opt, 5, "i", 1)) != (_VALID, 1, 1, _RELU, 1, 1):
            raise ValueError(f"conv {k}: options differ from VALID/1/1/ReLU")
    for k in (1, 3):                                   # Pool2DOptions: VALID, stride 2, 2x2
        opt = ops[k][3]
        if [F.scalar(opt, i, "b" if i == 0 else "i", 0) for i in range(5)] != [_VALID, 2, 2, 2, 2] or \
                F.scalar(opt, 5, "b", 0) != _NONE:
            raise ValueError(f"pool {k}: options differ from VALID 2x2/2")
    for k in (4, 5, 7):                                # no fused activation on MUL, ADD, FC
        if ops[k][3] is not None and F.scalar(ops[k][3], 0, "b", 0) != _NONE:
            raise ValueError(f"op {k}: unexpected fused activation")
    if ops[8][3] is not None and F.scalar(ops[8][3], 0, "f", 1.0) != 1.0:
        raise ValueError("softmax beta != 1")
    parts = [
        const(ops[0][1][1], (16, 3, 3, 1)), const(ops[0][1][2], (16,)),
        const(ops[2][1][1], (32, 3, 3, 16)), const(ops[2][1][2], (32,)),
        const(ops[4][1][1], (32,)), const(ops[5][1][1], (32,)),
        const(ops[7][1][1], (3, 64)), const(ops[7][1][2], (3,)),
    ]
    w = np.concatenate([a.reshape(-1) for a in parts]).astype(np.float32)
    assert w.size == WEIGHTS
    return w


class ColorClassifier:
    """The reference's ColorClassifier, served by the GPU. `model` is a .tflite path (the
    reference's ~model_path) or a packed float32 weight array."""

    def __init__(self, model, device: int = 0):
        from . import BatchEngine, load_params
        self.weights = np.ascontiguousarray(read_tflite(model) if isinstance(model, str) else model, np.float32)
        if self.weights.size != WEIGHTS:
            raise ValueError(f"{self.weights.size} weights, expected {WEIGHTS}")
        self._eng = BatchEngine(load_params("simulation"), device=device)   # a handle on `device`
        check(lib().cg_colornet_set(self._eng.handle, self.weights.ctypes.data, WEIGHTS))

    def classify(self, clouds, want_images=False):
        """clouds: list of (n_i, 4) float32 x, y, z, intensity, or PointCloud2 messages (read by
        field name like pc2.read_points). Returns (colors int32 (n,),
        probabilities float32 (n, 3), images uint8 (n, 15, 12) or None); colors use the negative
        codes SKIPPED / INDEX_ERROR / RANGE_ERROR where the reference skips or raises."""
        clouds = [c.xyzi() if hasattr(c, "xyzi") else c for c in clouds]
        n = len(clouds)
        offs = np.zeros(n + 1, np.uint32)
        for i, c in enumerate(clouds):
            offs[i + 1] = offs[i] + len(c)
        pts = np.ascontiguousarray(np.concatenate([np.asarray(c, np.float32).reshape(-1, 4) for c in clouds])
                                   if n and offs[-1] else np.zeros((1, 4), np.float32))
        colors = np.zeros(max(n, 1), np.int32)
        probs = np.zeros((max(n, 1), 3), np.float32)
        images = np.zeros((max(n, 1), 15, 12), np.uint8) if want_images else None
        check(lib().cg_classify_colors(self._eng.handle, pts.ctypes.data, offs.ctypes.data, n, colors.ctypes.data,
                                       probs.ctypes.data, images.ctypes.data if want_images else None))
        return colors[:n], probs[:n], (images[:n] if want_images else None)

    def handle_classify_color(self, cones_clouds):
        """The service handler (color_classifier_server.py:81-124): one colour per non-empty
        cloud, in request order. A cloud the reference's to_image cannot image raises as it does
        (ValueError from interp1d, IndexError from the image assignment)."""
        colors, _, _ = self.classify(cones_clouds)
        out = []
        for c in colors.tolist():
            if c == SKIPPED:
                continue
            if c == RANGE_ERROR:
                raise ValueError("A value in x_new is outside the interpolation range.")
            if c == INDEX_ERROR:
                raise IndexError("image row index out of bounds for axis 0 with size 15")
            out.append(c)
        return out

    __call__ = handle_classify_color


if __name__ == "__main__":
    # python -m cones_perception_amd.colornet dam_net.tflite dam_net.f32: the packed weights as
    # raw little-endian float32 (for C/C++ callers of cg_colornet_set)
    import sys
    read_tflite(sys.argv[1]).astype("<f4").tofile(sys.argv[2])
