#!/bin/bash
# GPU: pcl_sort probe (new vs a saved old build, if present), the PCL-order parity tests, a
# short bench with phase stamps. Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/pcl_probe 4000 243 || exit $?
timeout -k 10 60 ./tools/pcl_probe 300 1500 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_pcl_order.py tests/test_gpu_large.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_pcl.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_pcl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --stamps --no-cpu "$@" > gpurun_out/bench.log 2>&1 || exit $?
python tools/show_bench.py gpurun_out/bench.log | cut -c1-900
