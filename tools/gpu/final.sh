#!/bin/bash
# final checkpoint: full GPU suite, smoke, k-NN HBM counters (stamped), the default bench line, the
# same bench command under rocprofv3 --kernel-trace --stats, and the C3R8 line.  Stops at the
# first failing step.
set -o pipefail
out=gpurun_out/${1:-final}
mkdir -p "$out"
echo "[final] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
echo "[final] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
echo "[final] k-NN counters"
timeout -k 10 300 bash tools/knn_pmc.sh "$out/pmc" > "$out/pmc.log" 2>&1 || { tail -20 "$out/pmc.log"; exit 1; }
echo "[final] bench (default)"
timeout -k 10 400 python -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || { tail -20 "$out/bench_default.err"; exit 1; }
cat "$out/bench_default.json"
echo "[final] bench under rocprofv3"
root=$(pwd)
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$root/$out/prof" -o run -- python3 "$root/bench.py" --no-pmc > "$root/$out/bench_prof.json" 2> "$root/$out/bench_prof.err" ) || { tail -20 "$out/bench_prof.err"; exit 1; }
cat "$out/bench_prof.json"
echo "[final] bench C3R8"
timeout -k 10 300 python -u bench.py --workload C3R8 --no-cpu-baseline > "$out/bench_C3R8.json" 2> "$out/bench_C3R8.err" || { tail -20 "$out/bench_C3R8.err"; exit 1; }
cat "$out/bench_C3R8.json"
echo "[final] select counters"
timeout -k 10 400 bash tools/gpu/sel_counters.sh "$(basename $out)/sel" > "$out/sel.log" 2>&1 || { tail -20 "$out/sel.log"; exit 1; }
echo "[final] MLP counters"
timeout -k 10 400 bash tools/gpu/mlp_counters.sh "$(basename $out)/mlp" > "$out/mlp.log" 2>&1 || { tail -20 "$out/mlp.log"; exit 1; }
tail -3 "$out/mlp.log"
