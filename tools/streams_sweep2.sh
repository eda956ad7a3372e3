set -o pipefail
mkdir -p gpurun_out
for s in 3 4 2 3 4 5; do
  timeout -k 10 200 python bench.py --no-cpu --no-c5 --streams $s --steps 200 > gpurun_out/s$s.log 2>&1 || exit $?
  python -c "import json,sys; l=[json.loads(x) for x in open('gpurun_out/s$s.log') if x.startswith('{')][0]; print($s, round(l['value']/1e6,3), round(l['roofline']['frac'],3), round(l['roofline']['aggregate_frac'],3))"
done
