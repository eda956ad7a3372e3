"""GPU: C5 one frame per call, host enqueue time against the synchronised total (is the host
blocked inside the calls?), for the library CONES_GPU_LIB names (default: the in-tree one)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import cones_perception_amd as cp  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
params = cp.load_params("simulation")
raw = cp.synth_frames(1, first_frame=0, rings=128, cols=8192, clutter=60, cones_per_row=12)
d = torch.from_numpy(raw).cuda()
eng = cp.BatchEngine(params)
st = torch.cuda.Stream()
n = raw.shape[1] // 16
for _ in range(5):
    eng.run(d.data_ptr(), 1, n, 16, stream=st.cuda_stream)
st.synchronize()
calls = []
t0 = time.perf_counter()
for _ in range(reps):
    a = time.perf_counter()
    eng.run(d.data_ptr(), 1, n, 16, stream=st.cuda_stream)
    calls.append(time.perf_counter() - a)
t_enq = time.perf_counter() - t0
st.synchronize()
t_all = time.perf_counter() - t0
calls.sort()
print(f"per frame {t_all / reps * 1e6:.1f} us, enqueue {t_enq / reps * 1e6:.1f} us per call "
      f"(median {calls[len(calls) // 2] * 1e6:.1f}, max {calls[-1] * 1e6:.1f})")
