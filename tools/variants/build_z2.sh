#!/bin/bash
# Build the z2 NT-GEMM experiment (tools/variants/z2_nt.hip) into tools/variants/libz2_nt.so
set -e
cd "$(dirname "$0")"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form \
  -shared z2_nt.hip -o libz2_nt.so -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|Scratch|Occupancy" || true
test -f libz2_nt.so
