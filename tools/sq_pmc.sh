#!/bin/bash
# Usage (GPU box): tools/sq_pmc.sh <tag> <python script> [args] — SQ stall/issue counters per kernel.
set -e
root=$(pwd); tag=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM -d $root/gpurun_out/sq_$tag -o run -- python $root/"$@" > $root/gpurun_out/sq_$tag.log 2>&1
