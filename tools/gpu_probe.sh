#!/bin/bash
# GPU: the pcl_sort probe alone (per-step stamps of one case)
set -o pipefail
timeout -k 10 60 ./tools/pcl_probe 400 243 && timeout -k 10 60 ./tools/pcl_probe 50 1000 && timeout -k 10 60 ./tools/pcl_probe 50 60
