#!/bin/bash
# GPU iteration step (run through gpurun): parity suite, then the bench with phase stamps.
# Each GPU step has its own time limit; the bench only runs when the tests pass.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --stamps --no-cpu "$@" > gpurun_out/bench.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/bench.log | tail -4
exit $rc
