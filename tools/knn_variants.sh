#!/bin/bash
# Usage (GPU box): tools/knn_variants.sh <tag> — k-NN timings at the BASELINE sizes and variants.
set -e
out=$(pwd)/gpurun_out/knnvar_$1.txt
: > $out
for args in "--d 29 --kp1 31" "--d 47 --kp1 31" "--n 500000 --d 63 --kp1 51 --reps 2" "--n 20000 --d 2 --kp1 5"; do
  echo "== $args" >> $out
  timeout -k 10 120 python tools/knn_probe.py $args >> $out 2>&1
done
echo "== C3 sampled tau (S=16) + lists" >> $out
MEPOL_KNN_SAMPLE=16 MEPOL_KNN_FILTER=0 timeout -k 10 120 python tools/knn_probe.py >> $out 2>&1
echo done
