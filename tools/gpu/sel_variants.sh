#!/bin/bash
# select-kernel variants at C3 under rocprofv3: the select16_kernel row of each.
# Usage: tools/gpu/sel_variants.sh OUT LIB... (LIB = main or a libmepol_amd_<LIB>.so suffix)
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p "$out"
root=$(pwd)
for v in "$@"; do
  L=$root/mepol_amd/libmepol_amd.so; [ $v = main ] || L=$root/mepol_amd/libmepol_amd_$v.so
  ( cd /tmp && export TMPDIR=/tmp && MEPOL_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      -d "$root/$out/prof_$v" -o run -- python3 "$root/tools/knn_probe.py" --reps 2 $CFG \
      > "$root/$out/probe_$v.log" 2>&1 ) || { tail -20 "$out/probe_$v.log"; exit 1; }
  echo "== $v: $(grep 'knn ms' $out/probe_$v.log)"
  python3 tools/rocpd_stats.py "$out/prof_$v/run_results.db" 30 | grep select16 | cut -c1-40,100-160
done
