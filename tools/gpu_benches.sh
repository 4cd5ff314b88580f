#!/bin/bash
# Usage (on the GPU box): tools/gpu_benches.sh <tag> [workloads...]
# One bench line per workload (default C3 C4 C5 C2 C2S) plus a 2-rank rehearsal of C3; each step
# has its own time limit and the first failure ends the script.
set -e
tag=$1; shift
out=$(pwd)/gpurun_out
mkdir -p $out
wl=${@:-C3 C4 C5 C2 C2S}
for w in $wl; do
  if [ "$w" = "dp2" ]; then
    timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
      > $out/bench_${tag}_dp2.json 2> $out/bench_${tag}_dp2.err
  else
    timeout -k 10 400 python -u bench.py --workload $w > $out/bench_${tag}_$w.json 2> $out/bench_${tag}_$w.err
  fi
done
echo done
