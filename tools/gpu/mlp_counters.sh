#!/bin/bash
# SQ / TA / TD / LDS counters of the fused forward and dh1 + layer-1 backward at the C3 shapes
# (tools/mlp_kernels_once.py), one rocprofv3 --pmc pass per group.  Usage: tools/gpu/mlp_counters.sh OUT [LIB]
set -o pipefail
out=gpurun_out/$1; lib=${2:-}
mkdir -p "$out"
root=$(pwd)
L=$root/mepol_amd/libmepol_amd.so; [ -n "$lib" ] && L=$root/mepol_amd/libmepol_amd_$lib.so
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
           "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  MEPOL_AMD_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $grp -d "$root/$out/pmc$i" -o run -- \
    python3 "$root/tools/mlp_kernels_once.py" > "$root/$out/pmc$i.log" 2>&1 || echo "pass $i failed"
  (cd "$root" && python3 tools/pmc_table.py "$out/pmc$i/run_results.db" "e" 2>&1 | grep -A1 -E "policy_fwd|z2_head|layer1_kernel|dh1_layer1|wgrad_kernel") || true
done
