#!/bin/bash
# GPU iteration: full GPU parity suite (stops at the first failure), then bench sweeps.
# usage: tools/gpu_iter.sh "<stream counts>" [bench args]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/exp_sweep.sh base "${1:-1 3}" "${@:2}"
