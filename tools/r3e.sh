set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --no-cpu --no-c5"
timeout -k 10 200 $B --stamps --streams 1 > gpurun_out/r3e_stamps1.json 2>&1 || exit $?
timeout -k 10 200 $B --streams 4 --split-streams 2,1 > gpurun_out/r3e_s421.json 2>&1 || exit $?
timeout -k 10 200 $B --streams 3 > gpurun_out/r3e_s3.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu --c5 > gpurun_out/r3e_c5.json 2>&1 || exit $?
