#!/bin/bash
# round 4: a variant library's k-NN tests first (stop on failure), then probes main vs variant
set -o pipefail
out=gpurun_out/${1:-r4kv}; v=$2
mkdir -p $out
MEPOL_AMD_LIB=mepol_amd/libmepol_amd_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $out/knn_tests_$v.log 2>&1 || { tail -30 $out/knn_tests_$v.log; exit 1; }
tail -1 $out/knn_tests_$v.log
for rep in 1 2; do
for cfg in "" "--nq 25000" "--d 47" "--n 500000 --d 63 --kp1 51"; do
  for lib in main $v; do
    L=mepol_amd/libmepol_amd.so; [ $lib = main ] || L=mepol_amd/libmepol_amd_$lib.so
    echo "== $cfg $lib"
    MEPOL_AMD_LIB=$L timeout -k 10 120 python -u tools/knn_probe.py $cfg --reps 5 2>&1 | tail -1 || exit 1
  done
done
done | tee $out/probe.log
