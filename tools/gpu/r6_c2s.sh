#!/bin/bash
# Round 6: C2 / C2S lines and the C2S k-NN kernel split; C3 k-NN probe timing (probe-seed gate).
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
root=$(pwd)
for w in C2 C2S; do
  timeout -k 10 400 python -u bench.py --workload $w --no-cpu-baseline > "$out/bench_$w.json" 2> "$out/bench_$w.err" || { tail -20 "$out/bench_$w.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_$w.json')); print('$w', d['ms_per_step'], 'knn', d['knn_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$root/$out/prof_c2s" -o run -- python3 "$root/bench.py" --workload C2S --no-cpu-baseline --no-pmc > "$root/$out/prof_c2s.json" 2> "$root/$out/prof_c2s.err" || { tail -5 "$root/$out/prof_c2s.err"; exit 1; }
python3 "$root/tools/rocpd_stats.py" "$root/$out/prof_c2s/run_results.db" 14 | cut -c1-60,110-170
cd "$root"
timeout -k 10 120 python3 tools/knn_probe.py --reps 4 > "$out/c3_knn.log" 2>&1 && grep "knn ms" "$out/c3_knn.log"
