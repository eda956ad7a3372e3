#!/bin/bash
# GPU, one call: the large-path suites on the current default (lg_pq_flow with reserved children
# blocks and swap slots, LDS tasks for ranges of 2,049-4,096 records), then C5 interleaved
# against the level launches (lib_variants/levels) and the kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "large or pcl_order or hbm_leaves or route or rccl or tiled" > gpurun_out/r6_flow5_tests.log 2>&1 \
    || { echo "tests failed: $?"; grep -E "^E |FAILED|Timeout" gpurun_out/r6_flow5_tests.log | head -30; exit 1; }
echo "flow5: $(tail -1 gpurun_out/r6_flow5_tests.log)"
bash tools/c5_ab.sh notask levels 2>&1 | tee gpurun_out/r6_flow5_ab.txt || exit 1
bash tools/c5_profile.sh > gpurun_out/c5prof.out 2>&1 || { tail -20 gpurun_out/c5prof.out; exit 1; }
grep lg_pq_flow gpurun_out/c5prof_launches.txt; tail -1 gpurun_out/c5prof_launches.txt
CONES_GPU_LIB=$R/lib_variants/pqfst/libcones_gpu.so timeout -k 10 200 python -u tools/pqf_stamps.py > gpurun_out/pqf_stamps5.txt 2>&1 \
    || { tail -5 gpurun_out/pqf_stamps5.txt; exit 1; }
cat gpurun_out/pqf_stamps5.txt
