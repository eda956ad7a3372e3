#!/bin/bash
# GPU, one call: the large-path suites on the default (lg_pcl_leafmid: leaves and mid ranges in one
# launch), then C5 interleaved against the two-launch form (lib_variants/twolaunch) and the levels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "large or pcl_order or hbm_leaves or route or flow_edges or tiled" > gpurun_out/r6_leafmid_tests.log 2>&1 \
    || { echo "tests failed: $?"; grep -E "^E |FAILED|Timeout" gpurun_out/r6_leafmid_tests.log | head -30; exit 1; }
echo "leafmid: $(tail -1 gpurun_out/r6_leafmid_tests.log)"
bash tools/c5_ab.sh twolaunch 2>&1 | tee gpurun_out/r6_leafmid_ab.txt || exit 1
bash tools/c5_profile.sh > gpurun_out/c5prof.out 2>&1 || { tail -20 gpurun_out/c5prof.out; exit 1; }
tail -16 gpurun_out/c5prof_launches.txt
