#!/bin/bash
# An experiment build of ONE source with extra -D options, linked with every other object of the
# current build into rust-crdt_amd/libcrdt_gpu_<tag>.so; select it with CRDT_GPU_LIB=<path>.
#   scripts/build_variant.sh <tag> <source.hip> -DOPT=... [-DOPT2=...]
cd "$(dirname "$0")/../rust-crdt_amd" || exit 2
tag=$1; src=$2; shift 2
mkdir -p build_var_$tag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function "$@" -I../include -Icsrc -x hip -c csrc/$src -o build_var_$tag/$src.o || exit 1
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libcrdt_gpu_$tag.so $objs build_var_$tag/$src.o -ldl -Wl,-rpath,/opt/rocm/lib
