#!/bin/bash
# round 4: head backward prefetch depth / grid A/B (tools/head_probe.py per library)
set -o pipefail
out=gpurun_out/${1:-r4hp}; shift
mkdir -p $out
for v in main "$@"; do
  L=mepol_amd/libmepol_amd.so; [ $v = main ] || L=mepol_amd/libmepol_amd_$v.so
  echo "== $v"
  MEPOL_AMD_LIB=$L timeout -k 10 120 python -u tools/head_probe.py 2>&1 | grep head_bwd || exit 1
done | tee $out/head.log
