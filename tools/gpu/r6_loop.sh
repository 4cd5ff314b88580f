#!/bin/bash
# Round 6: device-loop / sharded parity tests, then the C3 and C3R8 timelines and bench lines.
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_gemm.py tests/test_gpu_policy.py tests/test_gpu_device_loop.py tests/test_gpu_sharded_graph.py tests/test_gpu_sharded_world2.py \
  tests/test_gpu_sharded_world2_distinct.py tests/test_gpu_reference_caller.py \
  tests/test_gpu_distributed.py > "$out/tests.log" 2>&1
rc=$?; tail -3 "$out/tests.log"; [ $rc = 0 ] || exit $rc
bash tools/gpu/timeline.sh "$1/tl" C3R8 || exit 1
for w in C3R8 C3 C3R8; do
  timeout -k 10 400 python -u bench.py --workload $w --no-cpu-baseline --no-pmc > "$out/bench_$w.json" 2> "$out/bench_$w.err" || { tail -20 "$out/bench_$w.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_$w.json')); print('$w', d['ms_per_step'], 'knn', d['knn_ms'])"
done
