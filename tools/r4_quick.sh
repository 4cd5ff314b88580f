#!/bin/bash
# round 4: selected GPU tests + bench lines (C3, C2) without the CPU baseline
set -o pipefail
out=gpurun_out/${1:-r4q}
shift
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -3 "$out/tests.log"
for w in C3 C2; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline \
    > "$out/bench_$w.json" 2> "$out/bench_$w.err" || { tail -20 "$out/bench_$w.err"; exit 1; }
  cat "$out/bench_$w.json"
done
