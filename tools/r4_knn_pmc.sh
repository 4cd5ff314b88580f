#!/bin/bash
# round 4: SQ counters of the C3 k-NN select (one pass per counter group)
set -o pipefail
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/${1:-r4pmc}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F16"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $out/p$i -o run -- \
    python3 $root/tools/knn_probe.py --reps 1 > $out/p$i.log 2>&1 || echo "pass $i failed rc=$?"
done
for f in $out/p*/run_results.db $out/p*/*/run_results.db; do
  [ -f "$f" ] && python3 $root/tools/pmc_table.py "$f" select16 >> $out/summary.txt
done
cat $out/summary.txt
