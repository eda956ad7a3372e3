set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_node.py tests/test_gpu_profiles.py tests/test_gpu_pcl_order.py tests/test_gpu_split_batch.py -v --timeout 120 --timeout-method thread > gpurun_out/r3f_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/r3f_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3f_bench.json 2>&1 || exit $?
