#!/bin/bash
# GPU: single-frame parity suites, C2 phase stamps, C2 latency (C++ node mirror).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_node.py tests/test_gpu_profiles.py tests/test_gpu_real_crops.py tests/test_gpu_sector_edges.py -v --timeout 120 --timeout-method thread > "$R/gpurun_out/r3k_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc" >> "$R/gpurun_out/r3k_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/c2_stamps.py 200 > "$R/gpurun_out/r3k_stamps.txt" 2>&1 || exit $?
for rep in 1 2; do timeout -k 10 60 "$R/cones_perception_amd/lib/nodes_demo" --latency 1000 >> "$R/gpurun_out/r3k_lat.txt" 2>&1 || exit $?; done
exit $rc
