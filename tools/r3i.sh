#!/bin/bash
# GPU: C5 kernel trace (per-launch durations of the large path) and a kernel trace of the C2
# C++ node mirror's latency loop.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
bash "$R/tools/c5_kernels.sh" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c2k" -o run \
  -- "$R/cones_perception_amd/lib/nodes_demo" --latency 300 > "$R/gpurun_out/c2k.log" 2>&1 || exit $?
