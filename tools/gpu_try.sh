#!/bin/bash
# usage: tools/gpu_try.sh OUTFILE TIMEOUT CMD  -- retries only while no GPU slot/box is free
out=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient" "$out" && ! grep -q "status=ok" "$out"; then sleep 150; continue; fi
  break
done
echo "final rc=$rc" >> "$out"
