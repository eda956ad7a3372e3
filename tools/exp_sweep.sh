#!/bin/bash
# GPU experiment: bench (no parity) for variant libraries over stream counts.
# usage: tools/exp_sweep.sh "<variant names, 'base' = default build>" "<stream counts>" [bench args]
set -o pipefail
mkdir -p gpurun_out
vars=$1; strs=$2; shift 2
for v in $vars; do
  if [ "$v" = base ]; then unset CONES_GPU_LIB; else export CONES_GPU_LIB=$PWD/lib_variants/$v/libcones_gpu.so; fi
  for s in $strs; do
    timeout -k 10 200 python bench.py --no-cpu --streams $s --steps 40 "$@" > gpurun_out/exp_${v}_s$s.log 2>&1 || { echo "fail $v $s"; tail -5 gpurun_out/exp_${v}_s$s.log; exit 1; }
    python -c "import json; l=[json.loads(x) for x in open('gpurun_out/exp_${v}_s$s.log') if x.startswith('{')][0]; r=l['roofline']; print('$v', $s, round(l['value']/1e6,3), 'Mfps', round(r['avg_kernel_ms']*1e3,1), 'us/launch', round(r['frac'],3), round(r['aggregate_frac'],3))"
  done
done
