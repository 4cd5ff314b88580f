#!/bin/bash
# Usage (on the GPU box): tools/knn_pmc.sh — HBM counters of the C3 k-NN call, one counter per pass.
set -e
root=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $root/gpurun_out/pmc_$c -o run -- \
    python $root/tools/knn_probe.py --reps 1 > $root/gpurun_out/pmc_$c.log 2>&1
done
