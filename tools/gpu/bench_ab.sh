#!/bin/bash
# bench lines under env A/B settings: tools/gpu/bench_ab.sh outdir workload VAR=a VAR=b
set -o pipefail
out=gpurun_out/${1:-r4bab}; w=$2; shift 2
mkdir -p "$out"
for rep in 1 2; do
  for kv in "$@"; do
    env "$kv" timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --steps 5 > "$out/b.json" 2> "$out/b.err" || { tail -20 "$out/b.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$out/b.json')); print('$w $kv', d['ms_per_step'], d.get('knn_ms'))"
  done
done
