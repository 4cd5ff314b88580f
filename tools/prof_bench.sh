#!/bin/bash
# Usage (on the GPU box): tools/prof_bench.sh <tag> [pytest targets...]
# Runs the given GPU tests, then a kernel-trace profile of a short bench into gpurun_out/prof_<tag>.
set -e
tag=$1; shift
root=$(pwd)
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -m pytest "$@" -x -q > gpurun_out/t_$tag.log 2>&1
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/prof_$tag -o run -- \
  python $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $root/gpurun_out/b_$tag.log 2>&1
