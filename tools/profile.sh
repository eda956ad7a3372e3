#!/bin/bash
# rocprofv3 evidence for profiles/ (run through gpurun from the repo root):
#   1. kernel trace + stats of the driver's bench command (--steps 20 --warmup 5, 3 streams, as
#      `value` is measured; the line's sustained pass follows the timed steps)
#   2. HBM traffic: FETCH_SIZE and WRITE_SIZE in separate --pmc passes, one stream
#   3. SQ issue/wait counters, one stream
#   4. the clock counters over the line's 200-step sustained pass (tools/clock_drift.py)
# Every step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof
rm -rf "$O" && mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {   # name, then the rocprofv3 arguments before "--"
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$O/$name" -o run -- \
        python3 "$R/bench.py" --no-cpu ${BENCH_ARGS:-} > "$O/$name.log" 2>&1 || { echo "step $name failed: $?"; exit 1; }
}
BENCH_ARGS="--steps 20 --warmup 5" run stats --kernel-trace --stats
BENCH_ARGS="--steps 5 --warmup 2 --streams 1" run fetch --pmc FETCH_SIZE
BENCH_ARGS="--steps 5 --warmup 2 --streams 1" run write --pmc WRITE_SIZE
BENCH_ARGS="--steps 5 --warmup 2 --streams 1" run sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD
BENCH_ARGS="--steps 20 --warmup 5 --no-c2 --no-c5" run clock --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
find "$O" -name "*.csv" | sort
