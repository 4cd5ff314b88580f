#!/bin/bash
# exit-crash hypothesis check: C2S under rocprofv3 with the rollout's cooperative launch off
# (MEPOL_ROLLOUT_MW=0: the one-workgroup form, a plain launch)
out=gpurun_out/${1:-segv_mw0}
mkdir -p "$out"
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
MEPOL_ROLLOUT_MW=0 SEGV_RUN_MAPS="$root/$out/maps.txt" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$root/$out/prof" -o run -- python3 "$root/tools/segv_run.py" "$root/bench.py" --workload C2S --steps 2 --no-cpu-baseline > "$root/$out/c2s.json" 2> "$root/$out/c2s.err"
echo "rocprofv3 C2S MW=0 rc=$?"
grep -v "^W2026\|^I2026" "$root/$out/c2s.err" | tail -30
exit 0
