#!/bin/bash
# round 4: the full GPU suite, verbose, one test per line (conftest names each test on stderr)
set -o pipefail
out=gpurun_out/${1:-r4}
mkdir -p "$out"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > "$out/gpu_tests.log" 2>&1
rc=$?
tail -5 "$out/gpu_tests.log"
exit $rc
