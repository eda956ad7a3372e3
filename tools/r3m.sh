#!/bin/bash
# GPU: large-frame parity suites, then the C5 kernel trace (tools/c5_kernels.sh) and bench's C5 leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_pcl_order.py tests/test_gpu_tiled.py tests/test_gpu_rccl.py -v --timeout 200 --timeout-method thread > "$R/gpurun_out/r3m_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc" >> "$R/gpurun_out/r3m_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash "$R/tools/c5_kernels.sh" || exit $?
for rep in 1 2; do timeout -k 10 120 python "$R/tools/c5_run.py" 200 >> "$R/gpurun_out/r3m_c5.txt" 2>&1 || exit $?; done
exit $rc
