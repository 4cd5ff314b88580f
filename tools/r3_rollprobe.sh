#!/bin/bash
# rollout phase probe (GridWorld C2 shape) and the C2 bench line
set -o pipefail
mkdir -p gpurun_out/rp
timeout -k 10 120 python3 -u tools/rollout_probe.py > gpurun_out/rp/probe.log 2>&1 &&
timeout -k 10 120 python3 -u tools/rollout_probe.py 20 1000 64 48 > gpurun_out/rp/probe_small.log 2>&1
echo rc=$?
