#!/bin/bash
# Round 6: one bench line per workload at HEAD (C3 with its CPU baseline; the others without).
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
for w in C3 C4 C5 C2 C2S C3R8 C4R8 C5R8; do
  extra="--no-cpu-baseline"; [ $w = C3 ] && extra=""
  timeout -k 10 500 python -u bench.py --workload $w $extra > "$out/bench_$w.json" 2> "$out/bench_$w.err" || { tail -20 "$out/bench_$w.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_$w.json')); print('$w', d['ms_per_step'], 'knn', d['knn_ms'], 'frac', d['roofline']['frac'], 'iters', d['config']['off_policy_iters'])"
done
