#!/bin/bash
# round 4: k-NN uneven first range A/B (MEPOL_KNN_FIRST percent); fallback counts in the probe line
set -o pipefail
out=gpurun_out/${1:-r4f}
mkdir -p "$out"
for cfg in "--d 29 --kp1 31" "--d 47 --kp1 31" "--n 500000 --d 63 --kp1 51" "--d 29 --kp1 31 --nq 25000"; do
  for f in 50 60 67 75; do
    echo "== $cfg first=$f"
    MEPOL_KNN_FIRST=$f timeout -k 10 120 python -u tools/knn_probe.py $cfg --reps 4 2>&1 | tail -1 || exit 1
  done
done | tee "$out/probe.log"
