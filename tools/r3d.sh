set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_split_batch.py tests/test_gpu_large.py -v --timeout 120 --timeout-method thread > gpurun_out/r3d_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/r3d_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python bench.py --steps 40 --warmup 5 --no-cpu --no-c5"
timeout -k 10 200 $B --stamps --streams 1 > gpurun_out/r3d_stamps1.json 2>&1 || exit $?
timeout -k 10 200 $B --streams 4 --split-streams 2,1 > gpurun_out/r3d_s421.json 2>&1 || exit $?
timeout -k 10 200 $B --streams 6 --split-streams 2,1 > gpurun_out/r3d_s621.json 2>&1 || exit $?
timeout -k 10 200 $B --streams 6 --split-streams 3,1 > gpurun_out/r3d_s631.json 2>&1 || exit $?
timeout -k 10 200 $B --streams 6 --split-streams 3,2 > gpurun_out/r3d_s632.json 2>&1 || exit $?
timeout -k 10 200 $B --streams 3 --fused > gpurun_out/r3d_fused.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --c5 > gpurun_out/r3d_c5.json 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3d_prof -o r3d -- python bench.py --steps 40 --warmup 5 --no-cpu --no-c5 --streams 4 --split-streams 2,1 > gpurun_out/r3d_prof.log 2>&1 || exit $?
