#!/bin/bash
# GPU, one call: the -m gpu suite and the default bench line (tools/gpu_quick.sh), the
# rocprofv3 evidence (tools/profile.sh), then the tiled C5 leg at one rank (bench.py --c5-tiled).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
tag=${1:-r4e}
bash tools/gpu_quick.sh $tag "large or single or done_word or staging" || exit $?
bash tools/profile.sh > gpurun_out/profile.out 2>&1 || { tail -20 gpurun_out/profile.out; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --steps 20 --c5-tiled > gpurun_out/${tag}_c5tiled.json 2> gpurun_out/${tag}_c5tiled.err || exit $?
