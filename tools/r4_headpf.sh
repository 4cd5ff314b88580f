#!/bin/bash
# round 4: head backward parity + prefetch depth A/B (tools/head_probe.py per library)
set -o pipefail
out=gpurun_out/${1:-r4hp}; shift
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_device_loop.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for v in main "$@"; do
  L=mepol_amd/libmepol_amd.so; [ $v = main ] || L=mepol_amd/libmepol_amd_$v.so
  echo "== $v"
  MEPOL_AMD_LIB=$L timeout -k 10 120 python -u tools/head_probe.py 2>&1 | grep head_bwd || exit 1
done | tee $out/head.log
