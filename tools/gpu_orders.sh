#!/bin/bash
# GPU: parity suite, then the default bench in both voxel orders (PCL default, point order).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for o in pcl point; do
  timeout -k 10 300 python bench.py --no-cpu --stamps --voxel-order $o > gpurun_out/bench_$o.log 2>&1 || exit $?
  echo "== $o"; python tools/show_bench.py gpurun_out/bench_$o.log | cut -c1-700; grep -o "\"c5_single_gpu\": {\"ms_per_frame\": [0-9.]*" gpurun_out/bench_$o.log; grep -o "\"single_frame\": {\"latency_ms\": [0-9.]*" gpurun_out/bench_$o.log
done
