#!/bin/bash
# GPU, one call: C3 A/B of pass 1's cache policy (lib_variants/nt1 = sc0, nt2 = nt) against the
# default (200-step bench runs, interleaved), then the rocprofv3 evidence (tools/profile.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r4_nt_ab.txt
: > "$out"
for r in 1 2; do
  for lib in default nt1 nt2; do
    if [ $lib = default ]; then L=""; else L=$R/lib_variants/$lib/libcones_gpu.so; fi
    CONES_GPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-c5 --steps 200 > gpurun_out/nt_${lib}_$r.log 2>&1 || exit 1
    python -c "import json; l=[json.loads(x) for x in open('gpurun_out/nt_${lib}_$r.log') if x.startswith('{')][0]; print('$lib run $r', round(l['value']/1e6,3), round(l['roofline']['frac'],3), round(l['roofline']['aggregate_frac'],3))" >> "$out" || exit 1
  done
done
cat "$out"
bash tools/profile.sh > gpurun_out/profile.out 2>&1 || { tail -20 gpurun_out/profile.out; exit 1; }
tail -3 gpurun_out/profile.out
