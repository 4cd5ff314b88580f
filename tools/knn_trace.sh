#!/bin/bash
# Usage (GPU box): tools/knn_trace.sh <tag> [probe args] — kernel-trace stats of the C3 k-NN call.
set -e
root=$(pwd); tag=$1; shift
mkdir -p $root/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $root/gpurun_out/kt_$tag -o run -- python $root/tools/knn_probe.py "$@" > $root/gpurun_out/kt_$tag.log 2>&1
