#!/bin/bash
# GPU, one call: the flow partition with its counters on separate lines and the cut folded into
# the per-range count (flow256 first through the large-path suites), then C5 frame times
# interleaved: the default level launches against 128 / 192 / 256-workgroup flow grids.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
CONES_GPU_LIB=$R/lib_variants/flow256/libcones_gpu.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 \
    --timeout-method thread -k "large or pcl_order or hbm_leaves or route" > gpurun_out/r6_flow3_tests.log 2>&1 \
    || { echo "flow256 tests failed: $?"; grep -E "^E |FAILED|Timeout" gpurun_out/r6_flow3_tests.log | head -30; exit 1; }
echo "flow256: $(tail -1 gpurun_out/r6_flow3_tests.log)"
bash tools/c5_ab.sh flow128 flow192 flow256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r6_flow3_ab.txt
