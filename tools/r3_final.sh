#!/bin/bash
# Round-3 final evidence (outputs under gpurun_out/fin/): GPU suite + smoke, bench lines for
# every workload (C3 with the CPU baseline), kernel-trace profiles of the C3 bench (one-rank and
# sharded at world 1), the k-NN HBM counters and the select kernel's SQ / TCC counters.
# Every step has its own time limit; the first failure ends the script.
set -e
R=$(pwd); out=$R/gpurun_out/fin; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $out/bench_C3.json 2> $out/bench_C3.err
for w in C4 C5 C2 C2S C3R8 C4R8 C5R8; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_$w.json 2> $out/bench_$w.err
done
MEPOL_BENCH_SHARDED=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_C3_sharded_w1.json 2> $out/bench_C3_sharded_w1.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/prof.log 2>&1
MEPOL_BENCH_SHARDED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_sharded -o run -- \
  python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $out/prof_sharded.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/pmc_$c -o run -- \
    python $R/tools/knn_probe.py --reps 1 > $out/pmc_$c.log 2>&1
done
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d $out/sq_knn -o run -- python $R/tools/knn_probe.py --reps 1 > $out/sq_knn.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d $out/tcc_knn -o run -- python $R/tools/knn_probe.py --reps 1 > $out/tcc_knn.log 2>&1
echo done
