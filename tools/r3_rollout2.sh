#!/bin/bash
# 4-wave multi-workgroup rollout: parity tests, phase probe, C2 / C2S bench lines
set -o pipefail
mkdir -p gpurun_out/rp2

timeout -k 10 120 python3 -u tools/rollout_probe.py > gpurun_out/rp2/probe.log 2>&1 &&
timeout -k 10 120 python3 -u tools/rollout_probe.py 20 1000 64 48 > gpurun_out/rp2/probe_small.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --workload C2 > gpurun_out/rp2/bench_C2.json 2> gpurun_out/rp2/bench_C2.err &&
timeout -k 10 300 python3 -u bench.py --workload C2S > gpurun_out/rp2/bench_C2S.json 2> gpurun_out/rp2/bench_C2S.err
echo rc=$?
