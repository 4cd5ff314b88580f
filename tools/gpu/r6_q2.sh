#!/bin/bash
# Round 6: two-query-tile select (select16q2_kernel) -- k-NN parity tests, then C3 / C3R8-shape
# timings: main (q2, occupancy 3, no accumulator pipelining), MEPOL_KNN_QT2=0 (one-tile
# kernel), q2o2p1 (occupancy 2, pipelined).
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
root=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_knn.py tests/test_gpu_knn_total.py > "$out/tests.log" 2>&1
rc=$?; tail -3 "$out/tests.log"; [ $rc = 0 ] || exit $rc
run() {  # name env lib nq
  MEPOL_AMD_LIB=$3 env $2 timeout -k 10 120 python3 tools/knn_probe.py --reps 4 --nq $4 > "$out/$1_$4.log" 2>&1 || { tail -5 "$out/$1_$4.log"; exit 1; }
  echo "$1 nq $4: $(grep 'knn ms' $out/$1_$4.log)"
}
for nq in 0 25000; do
  run q2 X=1 $root/mepol_amd/libmepol_amd.so $nq
  run old MEPOL_KNN_QT2=0 $root/mepol_amd/libmepol_amd.so $nq
  run q2o2p1 X=1 $root/mepol_amd/libmepol_amd_q2o2p1.so $nq
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$root/$out/prof" -o run -- \
  python3 "$root/tools/knn_probe.py" --reps 3 > "$root/$out/prof.log" 2>&1 || exit 1
python3 "$root/tools/rocpd_stats.py" "$root/$out/prof/run_results.db" 6 | awk -F, '{n=$1; sub(/\(.*/,"",n); printf "%-50s %s %s\n", substr(n,1,50), $2, $4}'
