#!/bin/bash
# Round 6: C3 / C3R8-shape k-NN call per split (probe seeds on; split 4 = XCD-pair ranges).
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
root=$(pwd)
for nq in 0 25000; do
  for sp in 2 4 8; do
    timeout -k 10 120 python3 tools/knn_probe.py --reps 4 --nq $nq --split $sp > "$out/nq${nq}_s$sp.log" 2>&1 || exit 1
    echo "nq $nq split $sp: $(grep 'knn ms' $out/nq${nq}_s$sp.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
for sp in 2 4; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$root/$out/prof$sp" -o run -- \
    python3 "$root/tools/knn_probe.py" --reps 3 --split $sp > "$root/$out/prof$sp.log" 2>&1 || exit 1
  echo "== split $sp"
  python3 "$root/tools/rocpd_stats.py" "$root/$out/prof$sp/run_results.db" 6 | awk -F, '{n=$1; sub(/\(.*/,"",n); printf "%-50s %s %s\n", substr(n,1,50), $2, $4}'
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$root/$out/pmcf$sp" -o run -- \
    python3 "$root/tools/knn_probe.py" --reps 1 --split $sp > "$root/$out/pmcf$sp.log" 2>&1 || { echo "pmc failed"; continue; }
  (cd "$root" && python3 tools/pmc_table.py "$out/pmcf$sp/run_results.db" select16 2>&1 | tail -1; python3 tools/pmc_table.py "$out/pmcf$sp/run_results.db" refine 2>&1 | tail -1) || true
done
