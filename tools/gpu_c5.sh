#!/bin/bash
# GPU, one call after a large-path change: the large-frame, PCL-order, tiled and RCCL suites
# (each frame bit for bit against the oracle), then the C5 frame's timing and kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
tag=${1:-c5}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "large or pcl or tiled or rccl or batch_queue" > gpurun_out/${tag}_tests.log 2>&1 \
    || { echo "tests failed: $?"; grep -E "^E |FAILED" gpurun_out/${tag}_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 120 python tools/c5_run.py 200 || exit $?
bash tools/c5_profile.sh > /dev/null || exit $?
head -1 gpurun_out/c5prof_gaps.txt
tail -1 gpurun_out/c5prof_launches.txt
