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
