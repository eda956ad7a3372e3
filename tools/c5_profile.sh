#!/bin/bash
# GPU: C5 large-path kernel trace (tools/c5_kernels.sh) and its per-frame summary
# (tools/c5_gaps.py, tools/c5_launches.py) into gpurun_out/c5prof_{gaps,launches}.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/c5_kernels.sh" || exit $?
python3 "$R/tools/c5_gaps.py" "$R/gpurun_out/c5k_default/run_kernel_trace.csv" > "$R/gpurun_out/c5prof_gaps.txt" || exit $?
python3 "$R/tools/c5_launches.py" "$R/gpurun_out/c5k_default/run_kernel_trace.csv" > "$R/gpurun_out/c5prof_launches.txt" || exit $?
cat "$R/gpurun_out/c5k_default.log"
