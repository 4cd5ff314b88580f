#!/bin/bash
# rollout after the ticket change: envs parity tests, then C2S under rocprofv3 (exit status and
# kernel stats), then the C2 / C2S bench lines
set -o pipefail
out=gpurun_out/${1:-roll}
mkdir -p "$out"
root=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_gpu_envs.py tests/test_gpu_full_entropy.py -x -v --timeout 200 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -40 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
( cd /tmp && export TMPDIR=/tmp && SEGV_RUN_MAPS="$root/$out/maps.txt" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$root/$out/prof" -o run -- python3 "$root/tools/segv_run.py" "$root/bench.py" --workload C2S --steps 2 --no-cpu-baseline > "$root/$out/c2s_prof.json" 2> "$root/$out/c2s_prof.err" )
rc=$?
echo "rocprofv3 C2S rc=$rc"
[ $rc -eq 0 ] || { grep -v "^W2026\|^I2026" "$out/c2s_prof.err" | tail -30; exit 1; }
python3 tools/rocpd_stats.py "$out/prof/run_results.db" 14 | cut -c1-150
for w in C2 C2S; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --no-cpu-baseline > "$out/bench_$w.json" 2> "$out/bench_$w.err" || { tail -20 "$out/bench_$w.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['ms_per_step'], 'knn', d.get('knn_ms'), 'rollout', d.get('rollout_ms'))"
done
