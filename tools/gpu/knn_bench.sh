#!/bin/bash
# k-NN parity tests, then the k-NN call at the bench shapes under rocprofv3 (per-kernel stats)
# and plain (HIP-event timing).  Usage: tools/gpu/knn_bench.sh OUT [LIB]
set -o pipefail
out=gpurun_out/${1:-knn}; lib=${2:-}
mkdir -p "$out"
root=$(pwd)
L=$root/mepol_amd/libmepol_amd.so; [ -n "$lib" ] && L=$root/mepol_amd/libmepol_amd_$lib.so
MEPOL_AMD_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_knn_total.py -x -q \
  --timeout 300 --timeout-method thread > "$out/knn_tests.log" 2>&1 || { tail -40 "$out/knn_tests.log"; exit 1; }
tail -1 "$out/knn_tests.log"
i=0
for cfg in "" "--nq 25000" "--d 47" "--n 500000 --d 63 --kp1 51"; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && MEPOL_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      -d "$root/$out/prof$i" -o run -- python3 "$root/tools/knn_probe.py" $cfg --reps 3 \
      > "$root/$out/probe_prof$i.log" 2>&1 ) || { tail -20 "$out/probe_prof$i.log"; exit 1; }
  echo "== $cfg (profiled)"; grep "knn ms" "$out/probe_prof$i.log"
  python3 tools/rocpd_stats.py "$out/prof$i/run_results.db" 4 | cut -c1-150
  MEPOL_AMD_LIB=$L timeout -k 10 120 python -u tools/knn_probe.py $cfg --reps 5 2>&1 | grep "knn ms" || exit 1
done
