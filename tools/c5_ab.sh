#!/bin/bash
# GPU: C5 frame time (tools/c5_run.py), the default library against variants (lib_variants/<name>),
# interleaved; with CHECK=1 each variant first runs the large-path suites against the oracle.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
for v in "$@"; do
  if [ "${CHECK:-0}" = 1 ]; then
    CONES_GPU_LIB=$R/lib_variants/$v/libcones_gpu.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
      --timeout 300 --timeout-method thread -k "large or pcl_order" > gpurun_out/ab_$v.log 2>&1 \
      || { echo "$v: tests failed"; grep -E "^E |FAILED" gpurun_out/ab_$v.log | head; exit 1; }
    echo "$v: $(tail -1 gpurun_out/ab_$v.log)"
  fi
done
for r in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then L=""; else L=$R/lib_variants/$v/libcones_gpu.so; fi
    echo -n "run $r $v: "
    CONES_GPU_LIB=$L timeout -k 10 120 python tools/c5_run.py 200 2>> gpurun_out/c5_ab.err || exit 1
  done
done
