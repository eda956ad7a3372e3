#!/bin/bash
# GPU: C2 through the C++ node mirror (nodes_demo --latency), staging helper threads 0 / 1 / 3,
# interleaved over three rounds, then the phase stamps of the split launch with the default pool.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for r in 1 2 3; do
  for k in 0 1 3; do
    echo -n "run $r threads $k: "
    CG_STAGE_THREADS=$k timeout -k 10 120 cones_perception_amd/lib/nodes_demo --latency 1000 | tail -1 || exit 1
  done
done
timeout -k 10 120 python tools/c2_stamps.py 200 || exit 1
