#!/bin/bash
# GPU, one call: the single-frame and tiled tests first (the split launch's done word, the
# one-slab halo), then C2 A/B (default against lib_variants/nodone: the C++ node mirror and the
# Python call), C5 A/B (default against lib_variants/nohint), the C5 kernel trace and the C2
# phase stamps. Outputs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "single or staging or tiled or split or pipeline" > gpurun_out/ab_first.log 2>&1 \
    || { echo "first step failed"; tail -40 gpurun_out/ab_first.log; exit 1; }
tail -3 gpurun_out/ab_first.log
out=gpurun_out/r4_ab.txt
: > "$out"
for r in 1 2; do
  for v in default nodone; do
    if [ $v = default ]; then L=""; LP=""; else L=$R/lib_variants/$v/libcones_gpu.so; LP=$R/lib_variants/$v; fi
    echo -n "C2 cpp $v run $r: " >> "$out"
    LD_LIBRARY_PATH=$LP timeout -k 10 60 cones_perception_amd/lib/nodes_demo --latency 3000 >> "$out" 2>&1 || exit 1
    CONES_GPU_LIB=$L timeout -k 10 150 python -c "
import bench, cones_perception_amd as cp
p = cp.load_params('simulation')
raw = cp.synth_frames(1, first_frame=0, rings=64, cols=1024)
s = bench.single_frame_latency(cp, p, raw, 0, reps=1000)
print('C2 python $v run $r:', round(s['latency_ms'] * 1e3, 1), 'us')" >> "$out" 2>&1 || exit 1
  done
done
for r in 1 2; do
  for v in default nohint; do
    if [ $v = default ]; then L=""; else L=$R/lib_variants/$v/libcones_gpu.so; fi
    echo -n "C5 $v run $r: " >> "$out"
    CONES_GPU_LIB=$L timeout -k 10 120 python3 tools/c5_run.py 100 >> "$out" 2>&1 || exit 1
  done
done
cat "$out"
bash tools/c5_profile.sh > /dev/null || exit 1
timeout -k 10 120 python3 tools/c2_stamps.py 200 > gpurun_out/c2_stamps.txt 2>&1 || exit 1
