#!/bin/bash
# GPU: does the 20-step timed region run below steady-state clocks? Interleaved bench runs
# with and without 300 ms of untimed steps before the warmup.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
for rep in 1 2 3; do
  for ph in 0 300; do
    echo -n "preheat $ph: " >> "$R/gpurun_out/r3l.txt"
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-c5 --preheat-ms $ph 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value']/1e6,3), round(d['ms_per_step'],4), round(d['roofline']['frac'],3))" >> "$R/gpurun_out/r3l.txt" || exit $?
  done
done
