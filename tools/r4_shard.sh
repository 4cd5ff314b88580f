#!/bin/bash
# round 4: sharded / device-loop tests, then C3R8 and C3 iteration timelines
set -o pipefail
out=gpurun_out/${1:-r4sh}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded_graph.py tests/test_gpu_device_loop.py tests/test_gpu_epoch.py tests/test_gpu_cli_multirank.py tests/test_gpu_bench_rehearsal.py tests/test_gpu_reference_caller.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
bash tools/r4_timeline.sh ${1:-r4sh} C3R8 && bash tools/r4_timeline.sh ${1:-r4sh} C3
