"""Diagnostic: ground-mode keep bits of the large path across runs vs host decisions."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cones_perception_amd as cp
from cones_perception_amd import _abi
import oracle_py as O
params = cp.load_params("simulation")
raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
msg = cp.frame_cloud(raw[0])
N = raw.shape[1] // 16
CH = 8192
P = raw[0].view(np.float32).reshape(-1, 4)
ol = O.lib()
sec = np.array([ol.oracle_sector(float(p[1]), float(p[0])) for p in P[:, :3]])
low = np.full(18, np.float32(-0.1), np.float32)
for s in range(17):
    zz = P[(sec == s), 2]
    zz = zz[~np.isnan(zz)]
    if zz.size: low[s] = min(low[s], zz.min())
T = np.array([np.nextafter(np.float32(np.float64(l) + 0.1), np.float32(np.inf)) if np.float64(np.float32(np.float64(l) + 0.1)) < np.float64(l) + 0.1 else np.float32(np.float64(l) + 0.1) for l in low], np.float32)
hostkeep = ~(P[:, 2].astype(np.float64) < (low[sec].astype(np.float64) + 0.1))
print("host K", int(hostkeep.sum()))
obj = cp.GroundRemover(params)
i = np.arange(N); c, r = i // CH, i % CH; k, ln = r // 512, r % 512
runs = []
for rep in range(6):
    out = obj.cloud_handler(msg)
    w = np.zeros((N // CH) * 512, np.uint64)
    _abi.check(_abi.lib().cg_debug_large_buffer(obj.handle, 2, w.ctypes.data, w.nbytes))
    bits = ((w[c * 512 + ln] >> k.astype(np.uint64)) & np.uint64(1)).astype(bool)
    runs.append(bits)
    print("run", rep, "K", out.n_kept, "bits", int(bits.sum()))
runs = np.array(runs)
bad = (runs != hostkeep[None, :]).any(0)
print("points differing from host:", int(bad.sum()))
for p in np.where(bad)[0][:12]:
    print("  point", p, "chunk", p // CH, "lane", (p % CH) % 512, "k", (p % CH) // 512, "z", P[p, 2], "sector", sec[p],
          "T", T[sec[p]], "host", bool(hostkeep[p]), "gpu", runs[:, p].astype(int).tolist())
