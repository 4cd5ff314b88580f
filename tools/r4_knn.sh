#!/bin/bash
# round 4: k-NN select gating A/B (MEPOL_KNN_GATE 1 | 4): parity tests, then timings
set -o pipefail
out=gpurun_out/${1:-r4k}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn.py -x \
  -m gpu -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 \
  || { tail -40 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for cfg in "--d 29 --kp1 31" "--d 47 --kp1 31" "--n 500000 --d 63 --kp1 51" "--d 29 --kp1 31 --nq 25000"; do
  for g in 1 4; do
    echo "== $cfg gate=$g"
    MEPOL_KNN_GATE=$g timeout -k 10 120 python -u tools/knn_probe.py $cfg --reps 4 2>&1 | tail -1 \
      || exit 1
  done
done | tee "$out/probe.log"
