#!/bin/bash
# short end-of-session confirmation: full GPU suite, smoke, the default bench line
set -o pipefail
out=gpurun_out/${1:-short}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -1 "$out/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 400 python -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || { tail -20 "$out/bench_default.err"; exit 1; }
cat "$out/bench_default.json"
