#!/bin/bash
# per-kernel times of tools/mlp_kernels_once.py under rocprofv3 for the product and variant libs
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
root=$(pwd)
for v in "$@"; do
  L=$root/mepol_amd/libmepol_amd.so; [ $v = main ] || L=$root/mepol_amd/libmepol_amd_$v.so
  ( cd /tmp && export TMPDIR=/tmp && MEPOL_AMD_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats \
      -d "$root/$out/prof_$v" -o run -- python3 "$root/tools/mlp_kernels_once.py" > "$root/$out/run_$v.log" 2>&1 ) || { tail "$out/run_$v.log"; exit 1; }
  echo "== $v"; python3 tools/rocpd_stats.py "$out/prof_$v/run_results.db" 4 | grep -E "policy_fwd|dh1_layer1" | cut -c1-60,110-170
done
