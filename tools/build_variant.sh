#!/bin/bash
# A/B builds: tools/build_variant.sh NAME EXTRA_FLAGS...  ->  mepol_amd/libmepol_amd_NAME.so
# (run the product against it with MEPOL_AMD_LIB=mepol_amd/libmepol_amd_NAME.so)
set -e
name=$1; shift
make -s -j8 BUILD=build_$name >/dev/null 2>&1 || true
mkdir -p build_v/$name
objs=()
for f in mepol_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  extra=""
  case $b in knn|knn_select_ks*) extra="-fno-honor-nans -mllvm -amdgpu-mfma-vgpr-form";; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result $extra "$@" -Iinclude -c $f -o build_v/$name/$b.o &
  objs+=(build_v/$name/$b.o)
  while [ $(jobs -r | wc -l) -ge 8 ]; do sleep 1; done
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o mepol_amd/libmepol_amd_$name.so "${objs[@]}"
echo built mepol_amd/libmepol_amd_$name.so
