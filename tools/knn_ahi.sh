#!/bin/bash
# A/B of the candidate-hi selection (MEPOL_KNN_AHI=1, default) vs split candidates (=0) at the
# BASELINE k-NN shapes, after the k-NN GPU tests.  Outputs under gpurun_out/knnahi/.
set -e
R=$(pwd); out=$R/gpurun_out/knnahi; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
for cfg in "C3:--n 200000 --d 29 --kp1 31" "C4:--n 200000 --d 47 --kp1 31" "C5:--n 500000 --d 63 --kp1 51"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for m in 1 0; do
    MEPOL_KNN_AHI=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_${name}_$m -o run -- python $R/tools/knn_probe.py --reps 3 $args > $out/probe_${name}_$m.log 2>&1
  done
done
echo done
