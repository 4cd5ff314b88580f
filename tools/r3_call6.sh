#!/bin/bash
set -e
R=$(pwd); out=$R/gpurun_out/c6; mkdir -p $out
for m in 0 1; do
  MEPOL_MAPPED_SCALARS=$m timeout -k 10 300 python -u tools/loop_debug.py C5 > $out/loop_C5_mapped$m.log 2>&1 || true
done
MEPOL_MAPPED_SCALARS=1 MEPOL_SPECULATE=0 timeout -k 10 300 python -u tools/loop_debug.py C5 > $out/loop_C5_mapped1_spec0.log 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_loop.py tests/test_gpu_sharded_graph.py tests/test_gpu_epoch.py tests/test_gpu_envs.py -x -q --timeout 300 --timeout-method thread > $out/tests_default.log 2>&1
for w in C2 C3R8 C5R8; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_$w.json 2> $out/bench_$w.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_C5R8 -o run -- \
  python $R/bench.py --workload C5R8 --steps 1 --warmup 1 --no-cpu-baseline > $out/prof_C5R8.log 2>&1
echo done
