#!/bin/bash
# f64 matrix-core / VALU issue-rate table (tools/f64_mfma_table.hip): timings, then the MFMA
# busy-cycle counters of the same binary in one --pmc pass.
set -o pipefail
out=gpurun_out/${1:-f64}
mkdir -p "$out"
root=$(pwd)
timeout -k 10 120 ./tools/f64_mfma_table > "$out/table.txt" 2>&1 || { tail "$out/table.txt"; exit 1; }
cat "$out/table.txt"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  -d "$root/$out/pmc" -o run -- "$root/tools/f64_mfma_table" > "$root/$out/pmc.log" 2>&1 || echo "pmc pass failed"
