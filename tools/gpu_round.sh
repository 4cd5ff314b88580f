#!/bin/bash
# Usage (on the GPU box): tools/gpu_round.sh <tag> [tests|bench|prof|pmc ...]
# Each step has its own time limit; the first failure ends the script.
set -e
tag=$1; shift
root=$(pwd)
out=$root/gpurun_out
mkdir -p $out
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > $out/tests_$tag.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.log 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py > $out/bench_$tag.json 2> $out/bench_$tag.err ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
        --output-format csv -d $out/prof_$tag -o run -- \
        python $root/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/profbench_$tag.log 2>&1) ;;
    clk)
      # effective clock of the f64 MFMA kernels and of the pure-MFMA probe (GRBM_GUI_ACTIVE is
      # summed over the 8 XCDs; MI355X_MICROARCH.md HBM/rocprofv3 section)
      for t in mlp:"python $root/tools/mlp_kernels_once.py" probe:"$root/tools/f64_rate_probe"; do
        name=${t%%:*}; cmd=${t#*:}
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE \
          SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_WAVE_CYCLES \
          --output-format csv -d $out/clk_$name -o run -- $cmd > $out/clk_$name.log 2>&1)
      done ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $c -d $out/pmc_$c -o run -- \
          python $root/tools/knn_probe.py --reps 1 > $out/pmc_$c.log 2>&1)
      done ;;
  esac
done
echo done
