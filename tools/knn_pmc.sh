#!/bin/bash
# Usage (on the GPU box): tools/knn_pmc.sh [outdir] -- HBM counters of the C3 k-NN call, one
# counter per pass, summarised into profiles/knn_pmc_C3.json (stamped with the k-NN source hash
# bench.py checks) and a copy under outdir.
set -e
root=$(pwd)
out=$root/${1:-gpurun_out}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/pmc_$c -o run -- \
    python3 $root/tools/knn_probe.py --reps 1 > $out/pmc_$c.log 2>&1
done
cd $root && python3 tools/knn_pmc_summary.py $out
