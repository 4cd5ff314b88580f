#!/bin/bash
# round 4: the remaining bench lines (no CPU baseline), one JSON per workload
set -o pipefail
out=gpurun_out/${1:-r4benches}
mkdir -p "$out"
for w in C4 C5 C2 C2S C4R8 C5R8; do
  echo "[benches] $w"
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > "$out/bench_$w.json" 2> "$out/bench_$w.err" || { tail -20 "$out/bench_$w.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_$w.json')); print('$w', d['ms_per_step'], d.get('knn_ms'))"
done
