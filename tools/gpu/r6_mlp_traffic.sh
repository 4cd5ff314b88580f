#!/bin/bash
# Round 6: HBM bytes of the iteration's f64 kernels (FETCH_SIZE and WRITE_SIZE, one counter per
# rocprofv3 pass) over tools/l1_probe.py (forward) and tools/dh1_ab.py (dh1 / dW2).
set -o pipefail
out=gpurun_out/$1; mkdir -p "$out"
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for prog in l1_probe dh1_ab; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$root/$out/${prog}_$c" -o run -- python3 "$root/tools/$prog.py" > "$root/$out/${prog}_$c.log" 2>&1 || exit 1
  done
done
echo done
