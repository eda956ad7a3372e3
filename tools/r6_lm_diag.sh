#!/bin/bash
# GPU: the 100k-point flow edge test under a variant library, with a short limit of its own.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
V=$1
CONES_GPU_LIB=$R/lib_variants/$V/libcones_gpu.so timeout -k 10 90 python -u -m pytest tests/test_gpu_flow_edges.py -x -v \
    --timeout 60 --timeout-method thread > gpurun_out/lmdiag_$V.log 2>&1 \
    || { echo "$V failed: $?"; grep -E "PASSED|FAILED|Timeout|^E " gpurun_out/lmdiag_$V.log | head; exit 1; }
echo "$V: $(tail -1 gpurun_out/lmdiag_$V.log)"
