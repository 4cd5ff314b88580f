#!/bin/bash
# the default bench command under rocprofv3 --kernel-trace --stats (kernel-time table)
set -o pipefail
out=gpurun_out/${1:-prof}
mkdir -p "$out"
root=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$root/$out/prof" -o run -- python3 "$root/bench.py" --no-pmc --no-cpu-baseline > "$root/$out/bench_prof.json" 2> "$root/$out/bench_prof.err" ) || { tail -20 "$out/bench_prof.err"; exit 1; }
cat "$out/bench_prof.json"
