#!/bin/bash
# GPU: a variant's large-path suites, then per-kernel C5 traces of the default library and the
# variant (tools/c5_kernels.sh), twice, summarised per launch (tools/c5_launches.py).
set -o pipefail
v=$1
CONES_GPU_LIB=lib_variants/$v/libcones_gpu.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "large or pcl_order or tiled or rccl" > gpurun_out/c5k_ab_$v.log 2>&1 \
  || { grep -E "^E |FAILED" gpurun_out/c5k_ab_$v.log | head; exit 1; }
tail -1 gpurun_out/c5k_ab_$v.log
for r in 1 2; do
  bash tools/c5_kernels.sh $v > /dev/null 2>&1 || exit 1
  python3 tools/c5_launches.py gpurun_out/c5k_default/run_kernel_trace.csv > gpurun_out/c5l_default_$r.txt || exit 1
  python3 tools/c5_launches.py gpurun_out/c5k_$v/run_kernel_trace.csv > gpurun_out/c5l_${v}_$r.txt || exit 1
done
