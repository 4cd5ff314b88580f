#!/bin/bash
# f64 MLP kernels: parity tests, then the C3 bench (epoch) on the product library and on a
# variant (mepol_amd/libmepol_amd_<V>.so), and the C3 bench under rocprofv3 for kernel times.
set -o pipefail
out=gpurun_out/${1:-mlp}; v=${2:-m16}
mkdir -p "$out"
root=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_policy.py tests/test_gpu_device_loop.py tests/test_gpu_entropy.py -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -40 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for lib in main $v main $v; do
  L=$root/mepol_amd/libmepol_amd.so; [ $lib = main ] || L=$root/mepol_amd/libmepol_amd_$lib.so
  MEPOL_AMD_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 > "$out/bench_$lib.json" 2> "$out/bench_$lib.err" || { tail -20 "$out/bench_$lib.err"; exit 1; }
  echo "$lib $(python3 -c "import json,sys; d=json.loads(open('$out/bench_$lib.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('knn_ms'), d.get('roofline_iteration', {}))")"
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$root/$out/prof" -o run -- python3 "$root/bench.py" --no-cpu-baseline --steps 2 > "$root/$out/bench_prof.json" 2> "$root/$out/bench_prof.err" ) || { tail -20 "$out/bench_prof.err"; exit 1; }
python3 tools/rocpd_stats.py "$out/prof/run_results.db" 12 | cut -c1-170
