#!/bin/bash
# GPU: host wait A/B (default hipStreamSynchronize against a variant, e.g. lib_variants/spin built
# with API_FLAGS=-DCG_SPIN_SYNC): C2 single-frame latency and the C5 single-GPU frame, interleaved.
set -o pipefail
mkdir -p gpurun_out
v=$1
for r in 1 2; do
  for lib in default $v; do
    if [ $lib = default ]; then L=""; else L=lib_variants/$lib/libcones_gpu.so; fi
    CONES_GPU_LIB=$L timeout -k 10 150 python -c "
import bench, cones_perception_amd as cp
p = cp.load_params('simulation')
raw = cp.synth_frames(1, first_frame=0, rings=64, cols=1024)
s = bench.single_frame_latency(cp, p, raw, 0, reps=500)
c = bench.c5_single_gpu(cp, p, 0, reps=200)
print('$lib run $r', 'C2', round(s['latency_ms'] * 1e3, 1), 'us', 'C5', round(c['ms_per_frame'] * 1e3, 1), 'us', c['V'], c['C'])" || exit $?
  done
done
