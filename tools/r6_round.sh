#!/bin/bash
# GPU round evidence in two calls (each under gpurun's limit):
#   tools/r6_round.sh A   smoke, the -m gpu suite (riskiest first), the default bench line
#   tools/r6_round.sh B   rocprofv3 evidence of the driver's command (tools/profile.sh), the C5
#                         kernel trace (launch count), the multi-rank harness (two gloo ranks sharing
#                         the GPU: C4 scatter and per-rank ingest), the tiled C5 leg at one rank
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
tag=${TAG:-r6}
mkdir -p gpurun_out
if [ "${1:-A}" = A ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.txt 2>&1 || { tail -20 gpurun_out/${tag}_smoke.txt; exit 1; }
  tail -1 gpurun_out/${tag}_smoke.txt
  bash tools/gpu_quick.sh $tag "large or single or done_word or staging or batch_fetch or c4" || exit $?
  python tools/show_bench.py gpurun_out/${tag}_bench.json || true
else
  bash tools/profile.sh > gpurun_out/profile.out 2>&1 || { tail -20 gpurun_out/profile.out; exit 1; }
  bash tools/c5_profile.sh > gpurun_out/c5prof.out 2>&1 || { tail -20 gpurun_out/c5prof.out; exit 1; }
  head -1 gpurun_out/c5prof_gaps.txt; tail -1 gpurun_out/c5prof_launches.txt
  CG_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-c5 \
      > gpurun_out/${tag}_gloo2.json 2> gpurun_out/${tag}_gloo2.err || { tail -20 gpurun_out/${tag}_gloo2.err; exit 1; }
  bash tools/c5_ab.sh levels 2>&1 | tee gpurun_out/r6_c5_final_ab.txt
  timeout -k 10 300 python bench.py --no-cpu --no-c2 --steps 5 --sustained-steps 0 --c5-tiled > gpurun_out/${tag}_c5tiled.json 2> gpurun_out/${tag}_c5tiled.err || { tail -20 gpurun_out/${tag}_c5tiled.err; exit 1; }
fi
