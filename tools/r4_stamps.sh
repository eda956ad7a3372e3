#!/bin/bash
# GPU, one call at HEAD: the C3 phase stamps under load (bench.py --stamps) and the C2 phase stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --no-c5 --steps 20 --stamps > gpurun_out/r4s_stamps.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/c2_stamps.py 200 > gpurun_out/r4s_c2_stamps.txt 2>&1 || exit $?
grep STAMPS gpurun_out/r4s_stamps.log | cut -c1-300
