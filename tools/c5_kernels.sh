#!/bin/bash
# GPU: per-kernel times of the C5 large path (rocprofv3 kernel trace of tools/c5_run.py), for
# the default library and optionally a variant (lib_variants/<name>).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for lib in default ${1:-}; do
  if [ $lib = default ]; then L=""; else L=$R/lib_variants/$lib/libcones_gpu.so; fi
  rm -rf "$R/gpurun_out/c5k_$lib"
  CONES_GPU_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c5k_$lib" -o run \
    -- python3 "$R/tools/c5_run.py" 100 > "$R/gpurun_out/c5k_$lib.log" 2>&1 || exit $?
done
