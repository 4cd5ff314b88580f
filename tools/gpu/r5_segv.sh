#!/bin/bash
# new parity tests, then ONE C2S bench under rocprofv3 with a native crash backtrace printer
set -o pipefail
out=gpurun_out/${1:-segv}
mkdir -p "$out"
root=$(pwd)
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_full_entropy.py tests/test_gpu_entropy.py tests/test_gpu_envs.py "tests/test_gpu_device_loop.py::test_unfused_mlp_kernels_match_fused" -x -v --timeout 200 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -40 "$out/tests.log"; exit 1; }
tail -3 "$out/tests.log"
cd /tmp && export TMPDIR=/tmp
SEGV_RUN_MAPS="$root/$out/maps.txt" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$root/$out/prof" -o run -- python3 "$root/tools/segv_run.py" "$root/bench.py" --workload C2S --steps 2 --no-cpu-baseline > "$root/$out/c2s.json" 2> "$root/$out/c2s.err"
rc=$?
echo "rocprofv3 C2S rc=$rc"
tail -60 "$root/$out/c2s.err"
exit 0
