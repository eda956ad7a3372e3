#!/bin/bash
# GPU, one call at HEAD: smoke(), the -m gpu suite and the default bench line (tools/gpu_quick.sh),
# then the multi-rank harness rehearsed with two gloo ranks sharing the box's GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
tag=${1:-r4f}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.txt 2>&1 || { tail -20 gpurun_out/${tag}_smoke.txt; exit 1; }
tail -1 gpurun_out/${tag}_smoke.txt
bash tools/gpu_quick.sh $tag "large or single or done_word or staging" || exit $?
CG_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-c5 \
    > gpurun_out/${tag}_gloo2.json 2> gpurun_out/${tag}_gloo2.err || { tail -20 gpurun_out/${tag}_gloo2.err; exit 1; }
tail -1 gpurun_out/${tag}_gloo2.json
# the PCL-order sort alone (one workgroup, LDS form, 243 records as C3's frames hold): its phase
# stamps, and 4,000 cases against libstdc++
timeout -k 10 120 cones_perception_amd/lib/pcl_probe 4000 243 > gpurun_out/${tag}_pcl_probe.txt 2>&1 || exit 1
timeout -k 10 120 cones_perception_amd/lib/pcl_probe 300 1500 >> gpurun_out/${tag}_pcl_probe.txt 2>&1 || exit 1
cat gpurun_out/${tag}_pcl_probe.txt
timeout -k 10 300 python bench.py --no-cpu --no-c2 --steps 5 --c5-tiled > gpurun_out/${tag}_c5tiled.json 2> gpurun_out/${tag}_c5tiled.err || exit 1
python -c "import json; l=[json.loads(x) for x in open('gpurun_out/${tag}_c5tiled.json') if x.startswith('{')][0]; t=l['c5_tiled']; print('c5', l['c5_single_gpu']['ms_per_frame'], l['c5_single_gpu']['point_order_ms_per_frame'], 'gather', t['gather']['ms_per_frame'], 'halo', t['halo']['ms_per_frame'], t['halo']['identical_to_single_gpu'])"
# C2: the split chunks prefetch their filter survivors during the arrival wait (default) against
# the library before it (lib_variants/c2base), C++ node mirror, interleaved
for r in 1 2; do
  for v in default c2base; do
    if [ $v = default ]; then LP=""; else LP=$R/lib_variants/$v; fi
    echo -n "C2 cpp $v run $r: "
    LD_LIBRARY_PATH=$LP timeout -k 10 60 cones_perception_amd/lib/nodes_demo --latency 3000 || exit 1
  done
done
