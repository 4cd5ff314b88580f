#!/bin/bash
# Round 6: k-NN parity tests with the current library, then C3 k-NN timings and the kernel split
# under rocprofv3 for the current library (new) and the A/B library $2 (old, MEPOL_AMD_LIB).
# Usage: tools/gpu/r6_knn_lib_ab.sh OUT ABLIB
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
root=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_knn.py tests/test_gpu_knn_total.py > "$out/tests.log" 2>&1
rc=$?; tail -3 "$out/tests.log"; [ $rc = 0 ] || exit $rc
for v in new old new old; do
  if [ $v = old ]; then export MEPOL_AMD_LIB=$root/$2; else unset MEPOL_AMD_LIB; fi
  timeout -k 10 120 python3 tools/knn_probe.py --reps 4 $CFG > "$out/$v.log" 2>&1 || exit 1
  echo "$v: $(grep 'knn ms' $out/$v.log)"
done
cd /tmp && export TMPDIR=/tmp
for v in ${ORDER:-new old}; do
  if [ $v = old ]; then export MEPOL_AMD_LIB=$root/$2; else unset MEPOL_AMD_LIB; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$root/$out/prof_$v" -o run -- \
    python3 "$root/tools/knn_probe.py" --reps 3 $CFG > "$root/$out/prof_$v.log" 2>&1 || exit 1
  echo "== $v"
  python3 "$root/tools/rocpd_stats.py" "$root/$out/prof_$v/run_results.db" 6 2>/dev/null | awk -F, '{print $1, $(NF-3)}' | cut -c1-40,100-
done
