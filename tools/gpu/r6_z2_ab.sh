#!/bin/bash
# Round 6: policy tests, then z2_head_kernel times at 200k and 25k rows (rocprofv3 stats over
# tools/l1_probe.py) and the C3 / C3R8 bench lines, for the current library (new) and the A/B
# library $2 (old, MEPOL_AMD_LIB).  Usage: tools/gpu/r6_z2_ab.sh OUT ABLIB
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
root=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_policy.py tests/test_gpu_device_loop.py > "$out/tests.log" 2>&1
rc=$?; tail -1 "$out/tests.log"; [ $rc = 0 ] || exit $rc
for v in new old; do
  if [ $v = old ]; then export MEPOL_AMD_LIB=$root/$2; else unset MEPOL_AMD_LIB; fi
  for n in 200000 25000; do
    ( cd /tmp && export TMPDIR=/tmp && L1_N=$n timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$root/$out/p_${v}_$n" -o run -- python3 "$root/tools/l1_probe.py" 20 > "$root/$out/p_${v}_$n.log" 2>&1 ) || exit 1
    echo "$v n=$n: $(python3 tools/rocpd_stats.py $out/p_${v}_$n/run_results.db 6 | grep -E 'z2_head|layer1_kernel' | awk -F, '{print $1, $(NF-3)}' | cut -c1-30,60-)"
  done
done
for v in new old new old; do
  if [ $v = old ]; then export MEPOL_AMD_LIB=$root/$2; else unset MEPOL_AMD_LIB; fi
  for w in C3 C3R8; do
    timeout -k 10 300 python3 bench.py --workload $w --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > "$out/bench_${v}_$w.json" 2> "$out/bench_${v}_$w.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" "$out/bench_${v}_$w.json" "$v $w"
  done
done
