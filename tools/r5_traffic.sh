#!/bin/bash
# GPU: where the frame kernel's HBM traffic goes. rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE (separate
# passes) of one-stream bench runs (5 steps) for the default library and variants that return after
# pass 1 (stop1), after pass 2 + the survivor gather (stop2) and after the pads and bounds (stop3),
# tools/variants/exp_stop.h. Summaries: gpurun_out/traffic/<lib>_<counter>.csv
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/traffic
rm -rf "$O" && mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for lib in ${LIBS:-default stop1 stop2 stop3}; do
  if [ $lib = default ]; then L=""; else L=$R/lib_variants/$lib/libcones_gpu.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    CONES_GPU_LIB=$L timeout -k 10 180 rocprofv3 --pmc $c --output-format csv -d "$O/${lib}_$c" -o run -- \
      python3 "$R/bench.py" --no-cpu --no-c5 --no-c2 --no-events --sustained-steps 0 --steps 5 --warmup 2 --streams 1 \
      > "$O/${lib}_$c.log" 2>&1 || { echo "$lib $c failed"; tail -5 "$O/${lib}_$c.log"; exit 1; }
  done
done
python3 "$R/tools/traffic_split.py" "$O"
