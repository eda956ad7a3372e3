set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_split_batch.py tests/test_gpu_pcl_order.py -v --timeout 200 --timeout-method thread > gpurun_out/r3c_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/r3c_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-c5 > gpurun_out/r3c_split.json 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-c5 --fused > gpurun_out/r3c_fused.json 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu --no-c5 > gpurun_out/r3c_split200.json 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c_prof -o r3c -- python bench.py --steps 40 --warmup 5 --no-cpu --no-c5 > gpurun_out/r3c_prof.log 2>&1 || exit $?
