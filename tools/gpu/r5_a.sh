#!/bin/bash
# round 5, call A: the whole GPU suite (incl. the total k-NN boundary), then the select's cost
# breakdown under rocprofv3 (product / loads+MFMA only / min tree without hits) and the
# exhaustive plan's speed at C3 size.
set -o pipefail
out=gpurun_out/${1:-r5a}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread \
  > "$out/gpu_tests.log" 2>&1 || { tail -60 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
root=$(pwd)
for v in main selp1 selp2; do
  L=$root/mepol_amd/libmepol_amd.so; [ $v = main ] || L=$root/mepol_amd/libmepol_amd_$v.so
  ( cd /tmp && export TMPDIR=/tmp && MEPOL_AMD_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      -d "$root/$out/prof_$v" -o run -- python3 "$root/tools/knn_probe.py" --reps 3 \
      > "$root/$out/probe_$v.log" 2>&1 ) || { tail -20 "$out/probe_$v.log"; exit 1; }
  tail -1 "$out/probe_$v.log"
done
for cfg in "--kp1 61" "--kp1 101" "--d 100" ; do
  echo "== exhaustive $cfg"
  timeout -k 10 200 python -u tools/knn_probe.py $cfg --reps 2 2>&1 | tail -2 || exit 1
done
