#!/bin/bash
# GPU, one call: the large-path suites on the 256-workgroup flow grid (more deferred swaps),
# C5 frame times interleaved (level launches = default, flow, flow256), the C4 test, and the C2
# staging-thread A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
CONES_GPU_LIB=$R/lib_variants/flow256/libcones_gpu.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 \
    --timeout-method thread -k "large or pcl_order or hbm_leaves or route" > gpurun_out/r6_flow256_tests.log 2>&1 \
    || { echo "flow256 tests failed: $?"; grep -E "^E |FAILED|Timeout" gpurun_out/r6_flow256_tests.log | head -30; exit 1; }
echo "flow256: $(tail -1 gpurun_out/r6_flow256_tests.log)"
bash tools/c5_ab.sh flow flow256 2>&1 | tee gpurun_out/r6_flow_ab.txt || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_c4.py -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r6_c4_test.log 2>&1 || { echo "c4 test failed: $?"; tail -30 gpurun_out/r6_c4_test.log; exit 1; }
tail -1 gpurun_out/r6_c4_test.log
bash tools/c2_ab.sh 2>&1 | tee gpurun_out/r6_c2_ab.txt
