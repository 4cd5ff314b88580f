#!/bin/bash
# round 4: one bench + kernel trace + iteration timeline under the given env (VAR=VAL ...)
# usage: tools/r4_tl_env.sh outdir workload VAR=VAL...
set -o pipefail
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/${1:-r4tl}
w=${2:-C2S}
shift 2
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o run -- python3 $root/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
f=$(ls $out/tr/*kernel_trace.csv $out/tr/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $root/tools/iteration_timeline.py $f > $out/timeline.txt && cat $out/timeline.txt
