#!/bin/bash
# GPU, one call: the partition cut computed in S4 (default) against the library before it
# (lib_variants/c2base): the sort probes against libstdc++, the -m gpu suite, then C3 (200-step
# bench runs) and C2 (C++ node mirror) interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r4_sortcut.txt
: > "$out"
timeout -k 10 120 cones_perception_amd/lib/pcl_probe 4000 243 >> "$out" 2>&1 || { cat "$out"; exit 1; }
timeout -k 10 120 cones_perception_amd/lib/pcl_probe 300 1500 >> "$out" 2>&1 || { cat "$out"; exit 1; }
timeout -k 10 120 cones_perception_amd/lib/pcl_leaf_probe 400 4096 9 >> "$out" 2>&1 || { cat "$out"; exit 1; }
bash tools/gpu_quick.sh sc "pcl or large or done_word" >> "$out" 2>&1 || { cat "$out"; exit 1; }
tail -2 gpurun_out/sc_gpu.log >> "$out"
for r in 1 2; do
  for v in default c2base; do
    if [ $v = default ]; then L=""; LP=""; else L=$R/lib_variants/$v/libcones_gpu.so; LP=$R/lib_variants/$v; fi
    CONES_GPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-c5 --steps 200 > gpurun_out/sc_${v}_$r.log 2>&1 || exit 1
    python -c "import json; l=[json.loads(x) for x in open('gpurun_out/sc_${v}_$r.log') if x.startswith('{')][0]; print('C3 $v run $r', round(l['value']/1e6,3), round(l['roofline']['aggregate_frac'],3), 'C2 py', round(l['single_frame']['latency_ms']*1e3,1))" >> "$out" || exit 1
    echo -n "C2 cpp $v run $r: " >> "$out"
    LD_LIBRARY_PATH=$LP timeout -k 10 60 cones_perception_amd/lib/nodes_demo --latency 3000 >> "$out" 2>&1 || exit 1
  done
done
cat "$out"
