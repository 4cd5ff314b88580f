#!/bin/bash
# k-NN selection with sampled per-query bounds and XCD-resident candidate ranges (split 8/16):
# one line per configuration (tools/knn_probe.py, C3 size).  Usage on the GPU box.
set -e
out=gpurun_out/knn_sweep.txt
: > $out
run() { echo "== $*" >> $out; env "$@" >> $out 2>&1; }
run timeout -k 5 60 python tools/knn_probe.py --reps 3
run timeout -k 5 60 python tools/knn_probe.py --reps 3 --split 8
for S in 8 16 32; do
  run MEPOL_KNN_SAMPLE=$S MEPOL_KNN_FILTER=0 timeout -k 5 60 python tools/knn_probe.py --reps 3 --split 8
done
run MEPOL_KNN_SAMPLE=16 MEPOL_KNN_FILTER=0 timeout -k 5 60 python tools/knn_probe.py --reps 3 --split 16
run MEPOL_KNN_SAMPLE=16 MEPOL_KNN_FILTER=0 timeout -k 5 60 python tools/knn_probe.py --reps 3 --split 4
run MEPOL_KNN_SAMPLE=16 MEPOL_KNN_FILTER=0 timeout -k 5 60 python tools/knn_probe.py --reps 3
echo done
