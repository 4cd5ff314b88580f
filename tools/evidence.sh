#!/bin/bash
# Round evidence on the GPU box: bench lines for every workload and a kernel-trace profile of
# the default bench.  Usage: tools/evidence.sh <tag>   (outputs under gpurun_out/ev_<tag>/)
set -e
tag=$1
R=$(pwd)
out=$R/gpurun_out/ev_$tag
mkdir -p $out
timeout -k 10 240 python -u bench.py > $out/bench_C3.json 2> $out/bench_C3.err
for w in C4 C5 C2 C2S; do
  timeout -k 10 240 python -u bench.py --workload $w --steps 3 --warmup 1 > $out/bench_$w.json 2> $out/bench_$w.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- \
  python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/prof.log 2>&1
