#!/bin/bash
# round 4: k-NN tests + probe shapes for the main library and A/B variant libraries (args)
set -o pipefail
out=gpurun_out/${1:-r4kl}; shift
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $out/knn_tests.log 2>&1 || { tail -30 $out/knn_tests.log; exit 1; }
tail -1 $out/knn_tests.log
for rep in 1 2; do
for cfg in "" "--nq 25000" "--d 47"; do
  for v in main "$@"; do
    L=mepol_amd/libmepol_amd.so; [ $v = main ] || L=mepol_amd/libmepol_amd_$v.so
    echo "== $cfg $v"
    MEPOL_AMD_LIB=$L timeout -k 10 120 python -u tools/knn_probe.py $cfg --reps 5 2>&1 | tail -1 || exit 1
  done
done
done | tee $out/probe.log
