#!/bin/bash
# round 4: k-NN parity (both merges) + timing of the refine merge variants and A/B libraries
set -o pipefail
out=gpurun_out/${1:-r4k5}; shift
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $out/knn_tests.log 2>&1 || { tail -30 $out/knn_tests.log; exit 1; }
tail -1 $out/knn_tests.log
MEPOL_KNN_RANK_MERGE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $out/knn_tests_rm1.log 2>&1 || { tail -30 $out/knn_tests_rm1.log; exit 1; }
tail -1 $out/knn_tests_rm1.log
for cfg in "" "--nq 25000" "--d 47" "--n 500000 --d 63 --kp1 51"; do
  for v in rm2 rm1 "$@"; do
    echo "== $cfg $v"
    L=mepol_amd/libmepol_amd.so; rm=2
    case $v in rm1) rm=1;; rm2) ;; *) L=mepol_amd/libmepol_amd_$v.so;; esac
    MEPOL_AMD_LIB=$L MEPOL_KNN_RANK_MERGE=$rm timeout -k 10 120 python -u tools/knn_probe.py $cfg --reps 4 2>&1 | tail -1 || exit 1
  done
done | tee $out/probe.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/tr3 -o run -- python3 tools/knn_probe.py --reps 2 > $out/tr3.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/tr -o run -- python3 tools/knn_probe.py --nq 25000 --reps 2 > $out/tr.log 2>&1 || exit 1
python3 tools/kstats.py $out/tr3/run_results.db 6
python3 tools/kstats.py $out/tr/run_results.db 6
