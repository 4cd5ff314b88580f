#!/bin/bash
# Round 6 probe: is the C3 select bound by the last partial round of workgroups?  Times the
# k-NN at query counts whose workgroup count is / is not a multiple of the co-resident slots,
# then L1/L2 counters of the select at C3.
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
root=$(pwd)
for nq in 196608 200000 184320 172032; do
  for sp in 0 1 3; do
    timeout -k 10 120 python3 tools/knn_probe.py --reps 4 --nq $nq --split $sp > "$out/nq${nq}_s$sp.log" 2>&1 || exit 1
    echo "nq $nq split $sp: $(grep 'knn ms' $out/nq${nq}_s$sp.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_REQ_sum TCC_READ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d "$root/$out/pmc$i" -o run -- \
    python3 "$root/tools/knn_probe.py" --reps 1 > "$root/$out/pmc$i.log" 2>&1 || { echo "pass $i failed"; continue; }
  (cd "$root" && python3 tools/pmc_table.py "$out/pmc$i/run_results.db" select16 2>&1) || true
done
