#!/bin/bash
# GPU: the single-frame suites on the default library, then C2 through the C++ node mirror
# (nodes_demo --latency 1000, 3 staging threads) for the default library against a variant
# (lib_variants/<name>/, with its own copy of nodes_demo so that $ORIGIN finds the variant),
# interleaved over four rounds; then the default's split-launch phase stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
V=${1:-c2base}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "single or done_word or staging or parity" > gpurun_out/c2ab_tests.log 2>&1 \
    || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/c2ab_tests.log | head; exit 1; }
echo "tests: $(tail -1 gpurun_out/c2ab_tests.log)"
for r in 1 2 3 4; do
  echo -n "run $r default: "; timeout -k 10 120 cones_perception_amd/lib/nodes_demo --latency 1000 | tail -1 || exit 1
  echo -n "run $r $V: "; timeout -k 10 120 lib_variants/$V/nodes_demo --latency 1000 | tail -1 || exit 1
done
timeout -k 10 120 python tools/c2_stamps.py 200 || exit 1
