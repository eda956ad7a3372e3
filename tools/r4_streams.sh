#!/bin/bash
# GPU, one call: C3 at 2, 3 and 4 streams (20-step bench runs, twice, interleaved), and pass 1
# with cache policy sc0 | nt (lib_variants/nt3) against the default nt. The variant libraries are
# built beforehand: tools/build_variant.sh nt3 -DCG_PASS1_AUX=3, stop1 -DCG_EXP_STOP=1,
# stop3 -DCG_EXP_STOP=3 (results: profiles/r4_streams_stop_ab.txt, r4_c5_fold_ab.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r4_streams.txt
: > "$out"
for r in 1 2; do
  for cfg in "3 default" "2 default" "4 default" "3 nt3"; do
    set -- $cfg
    if [ $2 = default ]; then L=""; else L=$R/lib_variants/$2/libcones_gpu.so; fi
    CONES_GPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-c5 --steps 20 --warmup 5 --streams $1 > gpurun_out/st_$1_$2_$r.log 2>&1 || exit 1
    python -c "import json; l=[json.loads(x) for x in open('gpurun_out/st_$1_$2_$r.log') if x.startswith('{')][0]; print('streams $1 $2 run $r', round(l['value']/1e6,3), round(l['roofline']['frac'],3), round(l['roofline']['aggregate_frac'],3))" >> "$out" || exit 1
  done
done
cat "$out"
# C5 after the decisions' fold went back to one workgroup: the large-path tests, the one-frame
# diagnostic and the kernel trace
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/st_large.log 2>&1 || { echo "large tests failed"; tail -30 gpurun_out/st_large.log; exit 1; }
tail -1 gpurun_out/st_large.log
for r in 1 2; do timeout -k 10 120 python3 tools/c5_diag.py 100 2>/dev/null || exit 1; done
bash tools/c5_profile.sh > /dev/null || exit 1
# where the time goes with the nt loads: builds that stop after pass 1 (stop1) and after the
# survivor gather (stop3), against the full kernel, 20 steps, interleaved
for r in 1 2; do
  for lib in default stop1 stop3; do
    if [ $lib = default ]; then L=""; else L=$R/lib_variants/$lib/libcones_gpu.so; fi
    CONES_GPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-c5 --no-c2 --steps 20 > gpurun_out/stop_${lib}_$r.log 2>&1 || exit 1
    python -c "import json; l=[json.loads(x) for x in open('gpurun_out/stop_${lib}_$r.log') if x.startswith('{')][0]; print('stop $lib run $r', round(l['value']/1e6,3), round(l['roofline']['frac'],3), round(l['roofline']['aggregate_frac'],3))" >> "$out" || exit 1
  done
done
cat "$out"
