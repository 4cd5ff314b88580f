#!/bin/bash
# Round 6: entropy / gamma parity tests, then C3 iteration timelines for the current library and
# the A/B libraries given as arguments (MEPOL_AMD_LIB=...).  Usage: r6_ent_ab.sh OUT LIB...
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p "$out"
root=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_entropy.py tests/test_gpu_full_entropy.py tests/test_gpu_device_loop.py \
  tests/test_gpu_sharded_world2_distinct.py > "$out/tests.log" 2>&1
rc=$?; tail -1 "$out/tests.log"; [ $rc = 0 ] || exit $rc
args=()
for l in "$@"; do args+=("MEPOL_AMD_LIB=$root/$l"); done
bash tools/gpu/timeline.sh "$(basename $out)/tl" C3 "${args[@]}" || exit 1
for f in $out/tl/timeline_C3_*.txt; do echo "== $f"; grep -E "gamma|entropy_fwd|iteration" $f | cut -c1-90; done
