#!/bin/bash
# GPU: parity of a variant library (tools/build_variant.sh), then a stream sweep of the bench.
# usage: tools/variant_check.sh <name> [streams...]
set -o pipefail
name=$1; shift
mkdir -p gpurun_out
export CONES_GPU_LIB=$PWD/lib_variants/$name/libcones_gpu.so
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/${name}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${name}_pytest.log; [ $rc -eq 0 ] || exit $rc
for s in "${@:-1 2 3}"; do
  timeout -k 10 200 python bench.py --no-cpu --streams $s --steps 40 > gpurun_out/${name}_s$s.log 2>&1 || exit $?
  python -c "import json; l=[json.loads(x) for x in open('gpurun_out/${name}_s$s.log') if x.startswith('{')][0]; r=l['roofline']; print('$name', $s, round(l['value']/1e6,3), round(r['frac'],3), round(r['aggregate_frac'],3))"
done
