#!/bin/bash
# GPU: the 131k-point detector frame alone under a variant library (default: lib_variants/notask),
# with a short limit of its own; then C5 frame times with that library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
V=${1:-notask}
CONES_GPU_LIB=$R/lib_variants/$V/libcones_gpu.so timeout -k 10 90 python -u -m pytest tests/test_gpu_large.py -x -v \
    --timeout 60 --timeout-method thread -k "detector" > gpurun_out/diag_$V.log 2>&1 \
    || { echo "$V detector failed: $?"; grep -E "^E |FAILED|Timeout" gpurun_out/diag_$V.log | head; exit 1; }
echo "$V: $(tail -1 gpurun_out/diag_$V.log)"
for r in 1 2; do
  echo -n "$V C5: "; CONES_GPU_LIB=$R/lib_variants/$V/libcones_gpu.so timeout -k 10 120 python tools/c5_run.py 200 2>> gpurun_out/c5_ab.err || exit 1
done
