#!/bin/bash
# Usage (GPU box): tools/knn_sq.sh <tag> — issue/stall and cache counters of the C3 k-NN call.
set -e
root=$(pwd); tag=$1
mkdir -p $root/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $root/gpurun_out/sq1_$tag -o run -- python $root/tools/knn_probe.py --reps 1 > $root/gpurun_out/sq1_$tag.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS -d $root/gpurun_out/sq2_$tag -o run -- python $root/tools/knn_probe.py --reps 1 > $root/gpurun_out/sq2_$tag.log 2>&1
python $root/tools/pmc_table.py $root/gpurun_out/sq1_$tag/run_results.db knn > $root/gpurun_out/sq_$tag.txt
python $root/tools/pmc_table.py $root/gpurun_out/sq2_$tag/run_results.db knn >> $root/gpurun_out/sq_$tag.txt
