#!/bin/bash
# GPU: C5 per-frame time (tools/c5_run.py) for the default library and variant builds
# (lib_variants/<name>), interleaved, two rounds; then the default library's kernel trace
# (tools/c5_profile.sh) and the C2 phase stamps (tools/c2_stamps.py).
#   tools/c5_ab.sh variant1 variant2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
out=$R/gpurun_out/c5_ab.txt
: > "$out"
for round in 1 2; do
  for v in default "$@"; do
    if [ "$v" = default ]; then L=""; else L=$R/lib_variants/$v/libcones_gpu.so; fi
    echo -n "$v round $round: " >> "$out"
    CONES_GPU_LIB=$L timeout -k 10 120 python3 "$R/tools/c5_run.py" 100 >> "$out" 2>&1 || exit 1
  done
done
cat "$out"
bash "$R/tools/c5_profile.sh" > /dev/null || exit 1
timeout -k 10 120 python3 "$R/tools/c2_stamps.py" 200 > "$R/gpurun_out/c2_stamps.txt" 2>&1 || exit 1
