#!/bin/bash
# GPU: the PCL-order workgroup sort alone (tools/pcl_probe, total time, no per-step stamps), the
# three-step level (shipped) against the four-step one (-DCG_PB_FOUR_STEP), interleaved, at C3's
# n = 243 and at 1,500 and 4,000 records; each probe checks its cases against libstdc++.
set -o pipefail
P=lib_variants/probe
for n in 243 1500 4000; do
  for r in 1 2 3; do
    for v in new old; do echo -n "n $n $v: "; timeout -k 10 60 $P/pcl_probe_$v 300 $n || exit $?; done
  done
done
