#!/bin/bash
# Round evidence on the GPU box: GPU test suite + smoke, bench lines for every workload, a
# kernel-trace profile of the default bench and the k-NN HBM counters.  Every step has its own
# time limit; the first failure ends the script.
# Usage: tools/evidence.sh <tag>   (outputs under gpurun_out/ev_<tag>/)
set -e
tag=$1
R=$(pwd)
out=$R/gpurun_out/ev_$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $out/bench_C3.json 2> $out/bench_C3.err
for w in C4 C5 C2 C2S C3R8; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 > $out/bench_$w.json 2> $out/bench_$w.err
done
timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
  > $out/bench_dp2_rehearsal.json 2> $out/bench_dp2_rehearsal.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/prof.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/pmc_$c -o run -- \
    python $R/tools/knn_probe.py --reps 1 > $out/pmc_$c.log 2>&1
done
echo done
