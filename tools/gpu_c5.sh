#!/bin/bash
# GPU: full parity suite, then a rocprofv3 kernel-stats run of C5's 1M-point frame.
set -o pipefail
mkdir -p gpurun_out/c5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c5 -o run -- python3 $R/tools/c5_run.py 20 > $R/gpurun_out/c5/log.txt 2>&1
rc=$?; grep C5 $R/gpurun_out/c5/log.txt; exit $rc
