#!/bin/bash
# GPU, one call: the done-word stress test (the default library, then lib_variants/presys, whose
# plain pack stores can be overtaken by the done word), C2 through the C++ node mirror, and the
# C5 enqueue diagnostic (tools/c5_diag.py) for the default library and the hint variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r4_c5c2.txt
: > "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log >> "$out"
CONES_GPU_LIB=$R/lib_variants/presys/libcones_gpu.so timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py \
    -k done_word -x -q --timeout 100 --timeout-method thread > gpurun_out/presys_doneword.log 2>&1
echo "presys done-word test rc=$? (1 = the stress test caught a stale pack)" >> "$out"
grep -m2 "AssertionError" gpurun_out/presys_doneword.log >> "$out"
for r in 1 2; do
  echo -n "C2 cpp default run $r: " >> "$out"
  timeout -k 10 60 cones_perception_amd/lib/nodes_demo --latency 3000 >> "$out" 2>&1 || exit 1
done
for r in 1 2; do
  for v in default base nohint nohintw; do
    if [ $v = default ]; then L=""; else L=$R/lib_variants/$v/libcones_gpu.so; fi
    echo -n "C5 $v run $r: " >> "$out"
    CONES_GPU_LIB=$L timeout -k 10 120 python3 tools/c5_diag.py 100 2>/dev/null >> "$out" || exit 1
  done
done
cat "$out"
