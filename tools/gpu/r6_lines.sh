#!/bin/bash
# Round 6: iteration timelines (C3, C3R8) and the other workloads' bench lines at HEAD.
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
bash tools/gpu/timeline.sh "$1/tl" C3 || exit 1
bash tools/gpu/timeline.sh "$1/tl" C3R8 || exit 1
for w in C5R8 C4 C5 C2 C2S; do
  timeout -k 10 400 python -u bench.py --workload $w --no-cpu-baseline > "$out/bench_$w.json" 2> "$out/bench_$w.err" || { tail -20 "$out/bench_$w.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_$w.json')); print('$w', d['ms_per_step'], 'knn', d['knn_ms'])"
done
