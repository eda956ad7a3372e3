#!/bin/bash
# GPU: the round's evidence at HEAD: full -m gpu suite, smoke(), the default bench line (with the
# CPU baseline), then tools/profile.sh (rocprofv3 kernel stats and PMC passes). Stops at the
# first failing step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_default.log | cut -c1-400
bash tools/profile.sh
