#!/bin/bash
# Round 6: GEMM/MLP parity tests, then dh1 (tools/dh1_ab.py) and the C3 bench line with the
# current library and with the A/B library in tools/variants/ab/ (MEPOL_AMD_LIB).
# Usage: tools/gpu/r6_gemm_ab.sh OUT ABLIB
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_gemm.py tests/test_gpu_policy.py tests/test_gpu_device_loop.py > "$out/tests.log" 2>&1
rc=$?; tail -3 "$out/tests.log"; [ $rc = 0 ] || exit $rc
for v in new old new old; do
  if [ $v = old ]; then export MEPOL_AMD_LIB=$(pwd)/$2; else unset MEPOL_AMD_LIB; fi
  timeout -k 10 120 python3 tools/dh1_ab.py > "$out/dh1_$v.log" 2>&1 || exit 1
  echo "$v: $(tail -2 $out/dh1_$v.log | tr '\n' ' ')"
done
for v in new old new old; do
  if [ $v = old ]; then export MEPOL_AMD_LIB=$(pwd)/$2; else unset MEPOL_AMD_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > "$out/bench_$v.json" 2> "$out/bench_$v.err" || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('knn_ms'))" "$out/bench_$v.json" $v
done
