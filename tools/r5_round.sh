#!/bin/bash
# GPU, one call: the -m gpu suite (riskiest first) and the default bench line (tools/gpu_quick.sh),
# the rocprofv3 evidence (tools/profile.sh), the multi-rank harness with two gloo ranks sharing
# the GPU, and the tiled C5 leg at one rank (RCCL group of one, collectives forced on).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
tag=${1:-r5}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.txt 2>&1 || { tail -20 gpurun_out/${tag}_smoke.txt; exit 1; }
tail -1 gpurun_out/${tag}_smoke.txt
bash tools/gpu_quick.sh $tag "large or single or done_word or staging or batch_fetch" || exit $?
python tools/show_bench.py gpurun_out/${tag}_bench.json || true
[ "${NO_PROFILE:-0}" = 1 ] || { bash tools/profile.sh > gpurun_out/profile.out 2>&1 || { tail -20 gpurun_out/profile.out; exit 1; }; }
CG_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-c5 \
    > gpurun_out/${tag}_gloo2.json 2> gpurun_out/${tag}_gloo2.err || { tail -20 gpurun_out/${tag}_gloo2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-c2 --steps 5 --sustained-steps 0 --c5-tiled > gpurun_out/${tag}_c5tiled.json 2> gpurun_out/${tag}_c5tiled.err || { tail -20 gpurun_out/${tag}_c5tiled.err; exit 1; }
