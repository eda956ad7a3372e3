#!/bin/bash
# Rebuild the in-tree libraries (no-op when current), then send one command to the GPU box.
#   tools/gpu_send.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; shift 2
cd "$(dirname "$0")/.." || exit 1
python cones_perception_amd/build.py > /tmp/gpu_send_build.log 2>&1 || { echo "build failed"; tail -20 /tmp/gpu_send_build.log; exit 1; }
exec /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
