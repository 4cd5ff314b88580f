#!/bin/bash
# Round-3 k-NN variants (LDS-staged candidate-hi default, 48-KB LDS variant, split-f16 register
# path) + the one-pass sharded iteration tests and the emulated per-rank bench.
set -e
R=$(pwd); out=$R/gpurun_out/c2; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -v --timeout 300 --timeout-method thread > $out/knn_tests.log 2>&1
MEPOL_KNN_LDS3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py -x -q --timeout 300 --timeout-method thread -k "config_sizes or edge or bitexact or split" > $out/knn_tests_lds3.log 2>&1
cd /tmp && export TMPDIR=/tmp
for cfg in "C3:--n 200000 --d 29 --kp1 31" "C4:--n 200000 --d 47 --kp1 31" "C5:--n 500000 --d 63 --kp1 51"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for v in "def:" "lds3:MEPOL_KNN_LDS3=1" "split:MEPOL_KNN_AHI=0"; do
    vn=${v%%:*}; ve=${v#*:}
    env $ve timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_${name}_$vn -o run -- python $R/tools/knn_probe.py --reps 3 $args > $out/probe_${name}_$vn.log 2>&1
  done
done
cd $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_envs.py tests/test_gpu_sharded_graph.py tests/test_gpu_distributed.py tests/test_gpu_cli_multirank.py tests/test_gpu_device_loop.py tests/test_gpu_gemm.py -x -v --timeout 300 --timeout-method thread > $out/sharded_tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload C3R8 --steps 2 --warmup 1 > $out/bench_C3R8.json 2> $out/bench_C3R8.err
MEPOL_BENCH_SHARDED=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_C3_sharded_w1.json 2> $out/bench_C3_sharded_w1.err
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/bench_C3.json 2> $out/bench_C3.err
timeout -k 10 300 python -u bench.py --workload C2 --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_C2.json 2> $out/bench_C2.err
echo done
