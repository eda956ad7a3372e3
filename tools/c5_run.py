"""GPU: the C5 single-GPU leg of bench.py alone (for rocprofv3 kernel traces of the large path)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import cones_perception_amd as cp  # noqa: E402

r = bench.c5_single_gpu(cp, cp.load_params("simulation"), 0, reps=int(sys.argv[1]) if len(sys.argv) > 1 else 50)
print(round(r["ms_per_frame"] * 1e3, 1), "us", r["V"], r["C"])
