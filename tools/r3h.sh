#!/bin/bash
# GPU: single-frame (split launch, staged input published per chunk) parity suites, then the
# default bench line (its single_frame leg is C2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_node.py tests/test_gpu_profiles.py tests/test_gpu_real_crops.py tests/test_gpu_sector_edges.py -v --timeout 120 --timeout-method thread > gpurun_out/r3h_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/r3h_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3h_bench.json 2> gpurun_out/r3h_bench.err || exit $?
exit $rc
