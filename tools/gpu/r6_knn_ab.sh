#!/bin/bash
# Round 6: k-NN parity tests, then C3 timings per MEPOL_KNN_SEED mode (and optional extra probe
# args in $CFG) with the kernel split under rocprofv3.
# Usage: tools/gpu/r6_knn_ab.sh OUT [tests]
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
root=$(pwd)
if [ "$2" = tests ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_knn.py tests/test_gpu_knn_total.py > "$out/tests.log" 2>&1
  rc=$?; tail -3 "$out/tests.log"; [ $rc = 0 ] || exit $rc
fi
for sd in ${SEEDS:-2 1}; do
  MEPOL_KNN_SEED=$sd timeout -k 10 120 python3 tools/knn_probe.py --reps 4 $CFG > "$out/seed$sd.log" 2>&1 || exit 1
  echo "seed $sd: $(grep 'knn ms' $out/seed$sd.log)"
done
cd /tmp && export TMPDIR=/tmp
for sd in ${SEEDS:-2 1}; do
  MEPOL_KNN_SEED=$sd timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$root/$out/prof$sd" -o run -- \
    python3 "$root/tools/knn_probe.py" --reps 3 $CFG > "$root/$out/prof$sd.log" 2>&1 || exit 1
  echo "== seed $sd"
  python3 "$root/tools/rocpd_stats.py" "$root/$out/prof$sd/run_results.db" 12 2>/dev/null | cut -c1-60,100-170 || \
    (cat "$root/$out/prof$sd/"*stats*.csv 2>/dev/null | head -12)
done
