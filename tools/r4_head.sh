#!/bin/bash
# GPU, one call at HEAD: smoke(), the -m gpu suite and the default bench line (20 steps).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
tag=${1:-r4h}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.txt 2>&1 || { tail -20 gpurun_out/${tag}_smoke.txt; exit 1; }
tail -1 gpurun_out/${tag}_smoke.txt | cut -c1-80
bash tools/gpu_quick.sh $tag "large or single or done_word or staging" || exit $?
