set -o pipefail
root=$(pwd); cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 3; do
  if [ $v = 0 ]; then unset MEPOL_AMD_LIB; else export MEPOL_AMD_LIB=$root/tools/variants/ab/libabl$v.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/abl/p$v" -o run -- python3 "$root/tools/knn_probe.py" --reps 3 > "$root/gpurun_out/abl/p$v.log" 2>&1 || exit 1
  echo "abl $v: $(python3 $root/tools/rocpd_stats.py $root/gpurun_out/abl/p$v/run_results.db 12 | grep refine_kernel | awk -F, '{print $(NF-3)}')"
done
