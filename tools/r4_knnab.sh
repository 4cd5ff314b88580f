#!/bin/bash
# round 4: k-NN GPU tests (default build) + probe shapes under env A/B settings given as args
# usage: tools/r4_knnab.sh outdir VAR=a VAR=b ...
set -o pipefail
out=gpurun_out/${1:-r4kab}; shift
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $out/knn_tests.log 2>&1 || { tail -30 $out/knn_tests.log; exit 1; }
tail -1 $out/knn_tests.log
for cfg in "" "--nq 25000" "--d 47" "--n 500000 --d 63 --kp1 51"; do
  for kv in "$@"; do
    echo "== $cfg $kv"
    env "$kv" timeout -k 10 120 python -u tools/knn_probe.py $cfg --reps 5 2>&1 | tail -1 || exit 1
  done
done | tee $out/probe.log
