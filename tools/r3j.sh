#!/bin/bash
# GPU: C2 latency of the C++ node mirror under the staging variants (CG_EXP_STAGE bit 0: pinned
# default staging memory instead of coherent; bit 1: copy before the launch, no per-chunk publish).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for rep in 1 2; do for m in 0 1 2 3; do
  echo -n "mode $m: " >> "$R/gpurun_out/r3j.txt"
  CG_EXP_STAGE=$m timeout -k 10 60 "$R/cones_perception_amd/lib/nodes_demo" --latency 1000 >> "$R/gpurun_out/r3j.txt" 2>&1 || exit $?
done; done
