#!/bin/bash
# Usage (GPU box): tools/knn_splits.sh <tag> — C3/C4 k-NN time vs candidate split.
out=$(pwd)/gpurun_out/knnsplit_$1.txt
: > $out
for d in 29 47; do
  for sp in 2 3 4 6 8 12 16; do
    echo "== d=$d split=$sp" >> $out
    timeout -k 10 120 python tools/knn_probe.py --d $d --split $sp >> $out 2>&1 || exit 1
  done
done
echo done
