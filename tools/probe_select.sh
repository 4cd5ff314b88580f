#!/bin/bash
# Usage (GPU box): tools/probe_select.sh <tag> <lib...> — per-kernel k-NN times per library build.
set -e
root=$(pwd); tag=$1; shift
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  MEPOL_AMD_LIB=$root/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/ps_${tag}_$n -o run -- python3 $root/tools/knn_probe.py --reps 1 ${PROBE_ARGS:-} > $root/gpurun_out/ps_${tag}_$n.log 2>&1
  echo "== $n"
  python3 $root/tools/rocpd_stats.py $root/gpurun_out/ps_${tag}_$n/run_results.db 8 | cut -c1-150
done
