#!/bin/bash
# GPU: the frame kernel's PCL-order sort. The probe against libstdc++ (4,000 cases, the wave form
# for n <= 256 and the workgroup form above), the sort alone at C3's n = 243 in both forms (total
# time, no per-step stamps), the parity suites, then the C3 phase stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
tag=${1:-srt}
L=cones_perception_amd/lib
timeout -k 10 120 $L/pcl_probe 4000 243 || exit $?
for r in 1 2 3; do
  for v in wave block; do echo -n "$v: "; timeout -k 10 60 $L/pcl_probe_$v 300 ${N:-243} || exit $?; done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "pcl or parity or profiles or node or single" > gpurun_out/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; grep -E "^E |FAILED" gpurun_out/${tag}_tests.log | head; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 200 python bench.py --no-cpu --no-c5 --steps 20 --warmup 5 --stamps > gpurun_out/${tag}_bench.log 2>&1 || exit $?
python tools/show_bench.py gpurun_out/${tag}_bench.log
