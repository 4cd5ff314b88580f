#!/bin/bash
# dh1 row-wave variants: the dh1 parity tests on each variant lib, then per-kernel times
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
root=$(pwd)
for v in "$@"; do
  L=$root/mepol_amd/libmepol_amd.so; [ $v = main ] || L=$root/mepol_amd/libmepol_amd_$v.so
  MEPOL_AMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > "$out/t_$v.log" 2>&1 || { tail -30 "$out/t_$v.log"; exit 1; }
  echo "$v: $(tail -1 $out/t_$v.log)"
done
bash tools/gpu/mlp_variants.sh "$(basename $out)" "$@"
