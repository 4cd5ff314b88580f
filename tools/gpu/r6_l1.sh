#!/bin/bash
# Round 6: layer1_kernel variants (RG row groups per wave) -- correctness (tools/fwd_check.py)
# and kernel times at C3 under rocprofv3.  Usage: tools/gpu/r6_l1.sh OUT LIB...
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p "$out"
root=$(pwd)
for v in "$@"; do
  L=$root/mepol_amd/libmepol_amd.so; [ $v = main ] || L=$root/mepol_amd/libmepol_amd_$v.so
  MEPOL_AMD_LIB=$L timeout -k 10 120 python3 tools/fwd_check.py > "$out/check_$v.log" 2>&1 || { tail "$out/check_$v.log"; exit 1; }
  echo "== $v"; head -3 "$out/check_$v.log" | cut -c1-110
  ( cd /tmp && export TMPDIR=/tmp && MEPOL_AMD_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats \
      -d "$root/$out/prof_$v" -o run -- python3 "$root/tools/l1_probe.py" 20 > "$root/$out/prof_$v.log" 2>&1 ) || exit 1
  python3 tools/rocpd_stats.py "$out/prof_$v/run_results.db" 4 | awk -F, '{n=$1; sub(/\(.*/,"",n); printf "%-45s %s %s %s\n", substr(n,1,45), $2, $4, $5}'
done
