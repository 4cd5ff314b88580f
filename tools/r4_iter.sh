#!/bin/bash
# round 4: entropy / device-loop tests, then the C3 iteration timeline
set -o pipefail
out=gpurun_out/${1:-r4it}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_entropy.py tests/test_gpu_device_loop.py tests/test_gpu_sharded_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
bash tools/r4_timeline.sh ${1:-r4it} C3
