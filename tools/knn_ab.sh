set -e
R=$(pwd); out=$R/gpurun_out/knnab; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
for m in 1 0; do
  MEPOL_KNN_RANK_MERGE=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof_m$m -o run -- python $R/tools/knn_probe.py --reps 3 > $out/probe_m$m.log 2>&1
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d $out/pmc_$c -o run -- python $R/tools/knn_probe.py --reps 1 > $out/pmc_$c.log 2>&1
done
echo done
