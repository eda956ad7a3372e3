#!/bin/bash
# GPU, one call: the large-path and PCL-order suites on each dataflow-partition variant
# (lib_variants/flow: lg_pq_flow; flowleaves: lg_pq_flow with the leaves and mid ranges inside),
# then C5 frame times interleaved against the default level launches, then the C4 test.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-flow flowleaves}; do
  CONES_GPU_LIB=$R/lib_variants/$v/libcones_gpu.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 \
      --timeout-method thread -k "large or pcl_order or hbm_leaves or route" > gpurun_out/r6_${v}_tests.log 2>&1 \
      || { echo "$v tests failed: $?"; grep -E "^E |FAILED|Timeout" gpurun_out/r6_${v}_tests.log | head -30; tail -5 gpurun_out/r6_${v}_tests.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r6_${v}_tests.log)"
done
bash tools/c5_ab.sh ${VARIANTS:-flow flowleaves} flow256 2>&1 | tee gpurun_out/r6_flow_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_c4.py -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r6_c4_test.log 2>&1 || { echo "c4 test failed: $?"; tail -30 gpurun_out/r6_c4_test.log; exit 1; }
tail -2 gpurun_out/r6_c4_test.log
