#!/bin/bash
# usage: tools/gpu_try.sh OUTFILE TIMEOUT CMD  -- retries only while no GPU slot/box is free
# (exit code 3, or a transient infrastructure failure), waiting out the back-off gpurun
# announces ("retry in Ns") before the next attempt; never after the command itself ran
out=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc = 3 ] || { grep -q "status=transient" "$out" && ! grep -q "status=ok" "$out"; }; then
    w=$(grep -o "retry in [0-9]*s" "$out" | tail -n1 | grep -o "[0-9]*")
    sleep $(( ${w:-150} + 15 ))
    continue
  fi
  break
done
echo "final rc=$rc" >> "$out"
