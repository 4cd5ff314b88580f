#!/bin/bash
# round 4: k-NN parity + timing (prune-bound seeding A/B) + select counters in one call
set -o pipefail
out=gpurun_out/${1:-r4k2}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -v --timeout 120 --timeout-method thread > $out/knn_tests.log 2>&1 || { tail -30 $out/knn_tests.log; exit 1; }
tail -2 $out/knn_tests.log
for cfg in "" "--nq 25000" "--d 47" "--n 500000 --d 63 --kp1 51"; do
  for sd in 1 0; do
    echo "== $cfg seed=$sd"
    MEPOL_KNN_SEED=$sd timeout -k 10 120 python -u tools/knn_probe.py $cfg --reps 4 2>&1 | tail -1 || exit 1
  done
done | tee $out/probe.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/tr -o run -- python3 tools/knn_probe.py --nq 25000 --reps 2 > $out/tr.log 2>&1 || exit 1
bash tools/r4_sel_pmc.sh ${1:-r4k2}/pmc
