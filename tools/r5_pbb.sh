#!/bin/bash
# GPU: the PCL-order workgroup sort alone (tools/pcl_probe, total time of case 0 and of all 300
# cases; the probe's arrays hold at most 2,048 records), the working tree's build (new) against
# HEAD's (old), interleaved, at 243, 1,000 and 2,000 records; each probe checks every case
# against libstdc++.
set -o pipefail
P=lib_variants/probe
for n in 243 1000 2000; do
  for r in 1 2; do
    for v in new old; do echo -n "n $n $v: "; timeout -k 10 60 $P/pcl_probe_$v 300 $n || exit $?; done
  done
done
