#!/bin/bash
# round 4: sharded / device-loop tests + the C3R8 line
set -o pipefail
out=gpurun_out/${1:-r4sh3}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded_graph.py tests/test_gpu_device_loop.py tests/test_gpu_epoch.py tests/test_gpu_cli_multirank.py tests/test_gpu_bench_rehearsal.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u bench.py --workload C3R8 --no-cpu-baseline > $out/bench_C3R8.json 2> $out/bench_C3R8.err || { tail -20 $out/bench_C3R8.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench_C3R8.json')); print('C3R8', d['ms_per_step'], d['knn_ms'])"
