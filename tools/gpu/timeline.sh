#!/bin/bash
# bench lines + kernel traces -> one off-policy iteration's timeline
# usage: tools/gpu/timeline.sh outdir workload [ENV=VAL ...]
set -o pipefail
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/${1:-r4t}
w=${2:-C3}
shift 2
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for kv in "" "$@"; do
  tag=${kv:-default}; tag=${tag##*/}; tag=${tag//=/_}
  ( [ -n "$kv" ] && export "$kv"; timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
    -d $out/tr_${w}_$tag -o run -- python3 $root/bench.py --workload $w --steps 2 --warmup 1 \
    --no-cpu-baseline > $out/bench_${w}_$tag.json 2> $out/bench_${w}_$tag.err ) \
    || { tail -20 $out/bench_${w}_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$out/bench_${w}_$tag.json')); print('$tag', d['ms_per_step'], d['knn_ms'], d['config']['off_policy_iteration'])"
  f=$(ls $out/tr_${w}_$tag/*kernel_trace.csv $out/tr_${w}_$tag/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 $root/tools/iteration_timeline.py $f > $out/timeline_${w}_$tag.txt && tail -1 $out/timeline_${w}_$tag.txt
done
