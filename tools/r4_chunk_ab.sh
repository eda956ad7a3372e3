#!/bin/bash
# GPU, one call: the chunked-batch parity tests (route 7), then C3 A/B (fused kernel against
# route 7, 200-step bench runs interleaved), then C2 and C5 against earlier libraries
# (lib_variants/base = 3ae0e8b, lib_variants/presys = f30d891). Outputs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunk_batch.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/chunk_tests.log 2>&1 || { echo "chunk tests failed"; tail -40 gpurun_out/chunk_tests.log; exit 1; }
tail -3 gpurun_out/chunk_tests.log
out=gpurun_out/r4_chunk_ab.txt
: > "$out"
for r in 1 2; do
  for route in 0 7; do
    timeout -k 10 200 python bench.py --no-cpu --no-c5 --steps 200 --route $route > gpurun_out/ab_route${route}_$r.log 2>&1 || exit 1
    python -c "import json; l=[json.loads(x) for x in open('gpurun_out/ab_route${route}_$r.log') if x.startswith('{')][0]; print('C3 route $route run $r', round(l['value']/1e6,3), round(l['roofline']['frac'],3), round(l['roofline']['aggregate_frac'],3), 'C2 py', round(l['single_frame']['latency_ms']*1e3,1), 'cpp', round(l['single_frame']['cpp_node']['latency_ms']*1e3,1))" >> "$out" || exit 1
  done
done
for r in 1 2; do
  for v in default base presys packfence; do
    if [ $v = default ]; then L=""; LP=""; else L=$R/lib_variants/$v/libcones_gpu.so; LP=$R/lib_variants/$v; fi
    echo -n "C2 cpp $v run $r: " >> "$out"
    LD_LIBRARY_PATH=$LP timeout -k 10 60 cones_perception_amd/lib/nodes_demo --latency 3000 >> "$out" 2>&1 || exit 1
  done
done
for r in 1 2; do
  for v in default base; do
    if [ $v = default ]; then L=""; else L=$R/lib_variants/$v/libcones_gpu.so; fi
    echo -n "C5 $v run $r: " >> "$out"
    CONES_GPU_LIB=$L timeout -k 10 120 python3 tools/c5_run.py 100 >> "$out" 2>&1 || exit 1
  done
done
cat "$out"
