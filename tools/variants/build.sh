#!/bin/bash
# Build libmepol_amd variants that differ in one source file: build.sh <name> <variant.hip> <replaced-object>
set -e
cd "$(dirname "$0")/../.."
name=$1; src=$2; rep=$3
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -Iinclude"
hipcc $FLAGS -c -x hip "$src" -o tools/variants/$name.o
objs=$(ls build/*.o | grep -v "build/$rep.o")
hipcc --offload-arch=gfx950 -shared -o tools/variants/$name.so $objs tools/variants/$name.o
echo built tools/variants/$name.so
