#!/bin/bash
# One GPU call after a kernel change: the riskiest tests first, each step under its own time
# limit, stopping at the first failure; then the whole -m gpu suite and the default bench line.
#   tools/gpu_quick.sh TAG "pytest -k expression for the first step"
tag=${1:-q}; sel=${2:-large}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$sel" \
    > gpurun_out/${tag}_first.log 2>&1 || { echo "first step failed: $?"; tail -30 gpurun_out/${tag}_first.log; exit 1; }
tail -3 gpurun_out/${tag}_first.log
bash tools/gpu_round.sh $tag
