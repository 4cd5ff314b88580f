#!/bin/bash
set -e
R=$(pwd); out=$R/gpurun_out/c5; mkdir -p $out
timeout -k 10 300 python -u tools/knn_repro.py > $out/knn_repro.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_loop.py tests/test_gpu_envs.py tests/test_gpu_sharded_graph.py -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || true
cd /tmp && export TMPDIR=/tmp
for cfg in "C3R8:--n 200000 --d 29 --kp1 31 --nq 25000" "C5R8:--n 500000 --d 63 --kp1 51 --nq 62500" "C2:--n 20000 --d 2 --kp1 5 --grid" "C2S:--n 24000 --d 2 --kp1 51 --grid" "C3:--n 200000 --d 29 --kp1 31"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_${name} -o run -- python $R/tools/knn_probe.py --reps 3 $args > $out/probe_${name}.log 2>&1
done
MEPOL_KNN_OCC3=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_C3_occ1 -o run -- python $R/tools/knn_probe.py --reps 3 > $out/probe_C3_occ1.log 2>&1
cd $R
for w in C3 C2 C2S C3R8 C5R8; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_$w.json 2> $out/bench_$w.err
done
echo done
