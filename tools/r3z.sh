set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3z_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/r3z_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3z_bench.json 2>&1 || exit $?
bash tools/profile.sh > gpurun_out/r3z_profile.log 2>&1 || exit $?
