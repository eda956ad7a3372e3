#!/bin/bash
# GPU, one call: the -m gpu suite (riskiest first), the default bench line (20 steps, as the
# driver runs it), the C3 phase stamps under load, the C2 phase stamps and the C5 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
tag=${1:-r4}
bash tools/gpu_quick.sh $tag "large or single or done_word or staging" || exit $?
timeout -k 10 200 python bench.py --no-cpu --no-c5 --steps 20 --stamps > gpurun_out/${tag}_stamps.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/c2_stamps.py 200 > gpurun_out/${tag}_c2_stamps.txt 2>&1 || exit $?
bash tools/c5_profile.sh > /dev/null || exit $?
