#!/bin/bash
# round 4: candidate-range split sweep with prune-bound seeding
set -o pipefail
out=gpurun_out/${1:-r4s2}
mkdir -p $out
for cfg in "" "--nq 25000" "--d 47"; do
  for sp in 0 2 3 4 6; do
    echo "== $cfg split=$sp"
    timeout -k 10 120 python -u tools/knn_probe.py $cfg --split $sp --reps 4 2>&1 | tail -2 || exit 1
  done
done | tee $out/splits.log
