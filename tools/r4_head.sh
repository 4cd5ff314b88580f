#!/bin/bash
# round 4: fused head backward parity + device-loop tests, then C3 / C3R8 bench lines
set -o pipefail
out=gpurun_out/${1:-r4h}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_device_loop.py tests/test_gpu_sharded_graph.py tests/test_gpu_entropy.py \
  tests/test_gpu_policy.py tests/test_gpu_reference_caller.py -m gpu -v --timeout 600 \
  --timeout-method thread > "$out/tests.log" 2>&1 || { tail -60 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
for w in C3 C3R8; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline \
    > "$out/bench_$w.json" 2> "$out/bench_$w.err" || { tail -20 "$out/bench_$w.err"; exit 1; }
  cat "$out/bench_$w.json"
done
