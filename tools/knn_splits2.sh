#!/bin/bash
out=$(pwd)/gpurun_out/knnsplit2_$1.txt
: > $out
for sp in 1 2; do
  echo "== d=29 split=$sp" >> $out; timeout -k 10 120 python tools/knn_probe.py --split $sp >> $out 2>&1 || exit 1
  for S in 8 16 32; do
    echo "== d=29 split=$sp sample=$S" >> $out
    MEPOL_KNN_SAMPLE=$S MEPOL_KNN_FILTER=0 timeout -k 10 120 python tools/knn_probe.py --split $sp >> $out 2>&1 || exit 1
  done
done
echo done
