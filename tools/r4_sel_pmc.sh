#!/bin/bash
# round 4: counters of the C3 select kernel (one rocprofv3 --pmc pass per group)
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/${1:-r4sp}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $out/p$i -o run -- python3 $root/tools/knn_probe.py --reps 1 > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; }
  python3 - $out/p$i/run_results.db <<'PY' || true
import sqlite3, sys, collections, glob
db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection").fetchall()
agg = collections.defaultdict(dict)
for d, n, cn, v in rows:
    if "select16" in n:
        agg[d][cn] = agg[d].get(cn, 0) + v
last = max(agg) if agg else None
if last is not None:
    for k, v in sorted(agg[last].items()):
        print(f"  {k:32s} {v:.4g}")
PY
done
