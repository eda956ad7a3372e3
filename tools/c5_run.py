"""Diagnostic: C5's 1,048,576-point dense frame through the large-frame path, `reps` times
(device-resident input), for rocprofv3 kernel traces of the global backend."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import cones_perception_amd as cp  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
params = cp.load_params("simulation")
raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
d = torch.from_numpy(raw).cuda()
eng = cp.BatchEngine(params)
st = torch.cuda.Stream()
n = raw.shape[1] // 16
for _ in range(3):
    eng.run(d.data_ptr(), 1, n, 16, stream=st.cuda_stream)
st.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    eng.run(d.data_ptr(), 1, n, 16, stream=st.cuda_stream)
st.synchronize()
dt = (time.perf_counter() - t0) / reps
r = eng.fetch(0)
print(f"C5 {dt * 1e3:.3f} ms/frame K={r.n_kept} M={r.n_filtered} V={r.voxels.shape[0]} C={r.centroids.shape[0]}")
