#!/bin/bash
# round 4: k-NN split sweep at C3 (200k queries) and the C3R8 per-rank shape (25k queries)
set -o pipefail
out=gpurun_out/${1:-r4s}
mkdir -p "$out"
for cfg in "--nq 25000" ""; do
  for s in 0 1 2 3 4 5 6 8 10 12 16; do
    echo "== $cfg split=$s"
    timeout -k 10 120 python -u tools/knn_probe.py --d 29 --kp1 31 $cfg --split $s --reps 4 2>&1 | tail -2 || exit 1
  done
done | tee "$out/splits.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_c3r8 -o run -- \
  python -u $GRAFT_REPO_ROOT/tools/knn_probe.py --d 29 --kp1 31 --nq 25000 --reps 4 > $GRAFT_REPO_ROOT/$out/prof_c3r8.log 2>&1
