#!/bin/bash
# One GPU call: the -m gpu suite, then (unless the suite ended in a fault, abort, timeout or
# hang) the default bench line and extra bench legs given as arguments.
#   tools/gpu_round.sh TAG [bench args for an extra leg ...]
# Outputs under gpurun_out/: TAG_gpu.log, TAG_bench.json/.err, TAG_extra.json/.err
tag=${1:-r3}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${tag}_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite ended with rc=$rc: no further GPU steps"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit $?
if [ $# -gt 0 ]; then
  timeout -k 10 300 python bench.py "$@" > gpurun_out/${tag}_extra.json 2> gpurun_out/${tag}_extra.err || exit $?
fi
exit $rc
