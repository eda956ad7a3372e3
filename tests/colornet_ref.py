"""CPU restatement of the colour classifier service (test infrastructure: the checker for
cg_classify_colors, never the product path).

to_image follows scripts/color_classifier_server.py:131-156 with numpy, as the reference does
(float64 angles, np.round half-to-even, negative row indices wrapping, interp1d([0,255],
[0,255]) raising outside its range, float -> uint8 by truncation, last write of a pixel
winning). The network follows the dam_net .tflite graph (CONV_2D/MAX_POOL_2D x2, MUL, ADD,
RESHAPE, FULLY_CONNECTED, SOFTMAX) in float64. The decision follows lines 112-116.

Parity status: the reference runs the network through TFLite, which is not importable here,
so the network's outputs are unpinned (float64 restatement, tolerance in the tests); the
weights are pinned to the reference's SavedModel checkpoint (tests/golden/make_dam_net.py)."""
import numpy as np

ROWS, COLS = 15, 12


class ImageError(Exception):
    pass


def to_image(pts):
    """(n, 4) float32 -> (15, 12) uint8, or raises IndexError / ValueError as the reference."""
    X, Y, Z, I = (pts[:, k].astype(np.float64) for k in range(4))
    vert = np.degrees(np.arctan2(Z, np.sqrt(pow(X, 2.0) + pow(Y, 2.0))))
    slope_vert = ROWS / (-15 - 15)
    rows = np.round(slope_vert * (vert - (-15))).astype(int)
    horiz = np.degrees(np.arctan2(Y, X))
    hmin, hmax = np.min(horiz), np.max(horiz)
    slope_h = (COLS - 1) / (hmax - hmin + 1e-16)
    cols = np.round(slope_h * (horiz - hmin)).astype(int)
    if np.any(I < 0) or np.any(I > 255):
        raise ValueError("A value in x_new is outside the interpolation range.")
    vals = I.copy()                                     # interp1d([0, 255], [0, 255]): identity
    image = np.zeros((ROWS, COLS, 1), np.uint8)
    image[rows, cols, 0] = vals                         # IndexError for rows outside [-15, 14]
    return image[:, :, 0]


def unpack(w):
    w = np.asarray(w, np.float64)
    k = 0

    def take(shape):
        nonlocal k
        n = int(np.prod(shape))
        a = w[k:k + n].reshape(shape)
        k += n
        return a
    p = dict(w1=take((16, 3, 3)), b1=take((16,)), w2=take((32, 3, 3, 16)), b2=take((32,)),
             bnm=take((32,)), bna=take((32,)), wd=take((3, 64)), bd=take((3,)))
    assert k == w.size
    return p


def forward(image, w):
    """dam_net on one (15, 12) image in float64 -> softmax probabilities (3,)."""
    p = unpack(w)
    x = image.astype(np.float64)
    c1 = np.zeros((13, 10, 16))
    for y in range(13):
        for xx in range(10):
            c1[y, xx] = np.einsum("okl,kl->o", p["w1"], x[y:y + 3, xx:xx + 3]) + p["b1"]
    c1 = np.maximum(c1, 0)
    p1 = c1[:12, :10].reshape(6, 2, 5, 2, 16).max(axis=(1, 3))
    c2 = np.zeros((4, 3, 32))
    for y in range(4):
        for xx in range(3):
            c2[y, xx] = np.einsum("oklc,klc->o", p["w2"], p1[y:y + 3, xx:xx + 3]) + p["b2"]
    c2 = np.maximum(c2, 0)
    p2 = c2[:4, :2].reshape(2, 2, 1, 2, 32).max(axis=(1, 3))
    flat = (p2 * p["bnm"] + p["bna"]).reshape(-1)      # (h, w, c) order
    lg = p["wd"] @ flat + p["bd"]
    e = np.exp(lg - lg.max())
    return e / e.sum()


def classify(clouds, w):
    """Per cloud: (colour or negative code as cg_classify_colors reports it, probabilities,
    image or None)."""
    out = []
    for c in clouds:
        c = np.asarray(c, np.float32).reshape(-1, 4)
        if c.shape[0] == 0:
            out.append((-1, np.zeros(3), None))
            continue
        try:
            img = to_image(c)
        except ValueError:
            out.append((-3, None, None))
            continue
        except IndexError:
            out.append((-2, None, None))
            continue
        pr = forward(img, w)
        col = int(np.argmax(pr)) + 1 if np.max(pr) >= 0.8 else 0
        out.append((col, pr, img))
    return out
