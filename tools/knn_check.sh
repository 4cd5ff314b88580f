#!/bin/bash
# k-NN parity tests, C3/C5 probe timings and the C3 HBM counters (outputs under gpurun_out/kc_<tag>/)
set -e
tag=$1; R=$(pwd); out=$R/gpurun_out/kc_$tag; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_entropy.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 120 python -u tools/knn_probe.py --reps 4 > $out/probe_C3.log 2>&1
timeout -k 10 200 python -u tools/knn_probe.py --n 500000 --d 63 --kp1 51 --reps 2 > $out/probe_C5.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python $R/tools/knn_probe.py --reps 2 > $out/prof.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/pmc_$c -o run -- python $R/tools/knn_probe.py --reps 1 > $out/pmc_$c.log 2>&1
done
echo done
