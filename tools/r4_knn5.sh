#!/bin/bash
# round 4: k-NN tests + C3 trace + select counters
set -o pipefail
out=gpurun_out/${1:-r4k7}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 120 --timeout-method thread > $out/knn_tests.log 2>&1 || { tail -30 $out/knn_tests.log; exit 1; }
tail -1 $out/knn_tests.log
timeout -k 10 120 python -u tools/knn_probe.py --reps 4 2>&1 | tail -1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/tr3 -o run -- python3 tools/knn_probe.py --reps 2 > $out/tr3.log 2>&1 || exit 1
python3 tools/kstats.py $out/tr3/run_results.db 5
bash tools/r4_sel_pmc.sh ${1:-r4k7}/pmc
