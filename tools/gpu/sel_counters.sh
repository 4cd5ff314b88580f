#!/bin/bash
# SQ / TA / TD counters of the C3 select kernel, one rocprofv3 --pmc pass per group (each well
# inside the per-block slot limits), summarised per kernel by tools/pmc_table.py.
# Usage: tools/gpu/sel_counters.sh OUT [LIB]
set -o pipefail
out=gpurun_out/$1; lib=${2:-}
mkdir -p "$out"
root=$(pwd)
L=$root/mepol_amd/libmepol_amd.so; [ -n "$lib" ] && L=$root/mepol_amd/libmepol_amd_$lib.so
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$root/$out/counters_list.txt" 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_WAVE32_LDS" \
           "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum" ; do
  i=$((i+1))
  MEPOL_AMD_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $grp -d "$root/$out/pmc$i" -o run -- \
    python3 "$root/tools/knn_probe.py" --reps 1 > "$root/$out/pmc$i.log" 2>&1 || echo "pass $i failed"
  (cd "$root" && python3 tools/pmc_table.py "$out/pmc$i/run_results.db" select16 2>&1) || true
done
