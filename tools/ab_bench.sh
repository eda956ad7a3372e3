# GPU: A/B of the default library against a variant (lib_variants/<name>), bench interleaved.
set -o pipefail
mkdir -p gpurun_out
v=$1; shift
for r in 1 2; do
  for lib in default $v; do
    if [ $lib = default ]; then L=""; else L=lib_variants/$lib/libcones_gpu.so; fi
    CONES_GPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-c5 --steps 200 "$@" > gpurun_out/ab_${lib}_$r.log 2>&1 || exit $?
    python -c "import json; l=[json.loads(x) for x in open('gpurun_out/ab_${lib}_$r.log') if x.startswith('{')][0]; print('$lib run $r', round(l['value']/1e6,3), round(l['roofline']['frac'],3), round(l['roofline']['aggregate_frac'],3))"
  done
done
