# GPU: frames/s against the number of streams, with the process's hardware queue count
# (GPU_MAX_HW_QUEUES, default 4) as the first argument.
set -o pipefail
mkdir -p gpurun_out
q=$1; shift
for s in "$@"; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu --no-c5 --streams $s --steps 200 > gpurun_out/q${q}_s$s.log 2>&1 || exit $?
  python -c "import json,sys; l=[json.loads(x) for x in open('gpurun_out/q${q}_s$s.log') if x.startswith('{')][0]; print('queues $q streams $s', round(l['value']/1e6,3), round(l['roofline']['frac'],3), round(l['roofline']['aggregate_frac'],3))"
done
