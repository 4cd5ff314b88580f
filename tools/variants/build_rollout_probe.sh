#!/bin/bash
# Builds the instrumented rollout kernel (diagnostic, not part of the product ABI) into
# tools/variants/librollout_probe.so
set -e
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -shared \
  -I mepol_amd/csrc tools/variants/rollout_probe.hip -o tools/variants/librollout_probe.so
echo built tools/variants/librollout_probe.so
