#!/bin/bash
# Builds the DPP VALU GEMM experiment (not part of the product ABI) into tools/variants/libdpp_gemm.so
set -e
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -shared \
  tools/variants/dpp_gemm.hip -o tools/variants/libdpp_gemm.so
echo built tools/variants/libdpp_gemm.so
