#!/bin/bash
# GPU: variants' large-path suites, then per-kernel C5 traces of the default library and each
# variant (tools/c5_kernels.sh), twice, summarised per launch (tools/c5_launches.py) into
# gpurun_out/c5l_<lib>_<round>.txt.
set -o pipefail
for v in "$@"; do
  CONES_GPU_LIB=lib_variants/$v/libcones_gpu.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "large or pcl_order or tiled or rccl" > gpurun_out/c5k_ab_$v.log 2>&1 \
    || { grep -E "^E |FAILED" gpurun_out/c5k_ab_$v.log | head; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c5k_ab_$v.log)"
done
for r in 1 2; do
  for v in "$@"; do
    bash tools/c5_kernels.sh $v > /dev/null 2>&1 || exit 1
    python3 tools/c5_launches.py gpurun_out/c5k_default/run_kernel_trace.csv > gpurun_out/c5l_default_${v}_$r.txt || exit 1
    python3 tools/c5_launches.py gpurun_out/c5k_$v/run_kernel_trace.csv > gpurun_out/c5l_${v}_$r.txt || exit 1
  done
done
