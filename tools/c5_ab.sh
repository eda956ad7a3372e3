#!/bin/bash
# GPU: C5 single-GPU frame time of the default library against a variant (lib_variants/<name>),
# interleaved, 200 frames per run.
set -o pipefail
mkdir -p gpurun_out
v=$1
for r in 1 2; do
  for lib in default $v; do
    if [ $lib = default ]; then L=""; else L=lib_variants/$lib/libcones_gpu.so; fi
    CONES_GPU_LIB=$L timeout -k 10 120 python -c "
import bench, cones_perception_amd as cp
r = bench.c5_single_gpu(cp, cp.load_params('simulation'), 0, reps=200)
print('$lib run $r', round(r['ms_per_frame'] * 1e3, 1), 'us', r['V'], r['C'])" || exit $?
  done
done
