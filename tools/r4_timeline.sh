#!/bin/bash
# round 4: C3 / C3R8 bench lines + kernel traces -> one off-policy iteration's timeline
set -o pipefail
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/${1:-r4t}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for w in C3 C3R8; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/tr_$w -o run -- \
    python3 $root/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline \
    > $out/bench_$w.json 2> $out/bench_$w.err || { tail -20 $out/bench_$w.err; exit 1; }
  cat $out/bench_$w.json
  f=$(ls $out/tr_$w/*kernel_trace.csv $out/tr_$w/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $root/tools/iteration_timeline.py $f > $out/timeline_$w.txt && tail -3 $out/timeline_$w.txt
done
