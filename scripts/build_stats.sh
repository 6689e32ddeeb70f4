#!/bin/bash
# Instrumented build (-DMAP_STATS: per-key phase cycles printed by map_fold_kernel) into
# rust-crdt_amd/libcrdt_gpu_stats.so; select it with CRDT_GPU_LIB=<path> (results unchanged).
cd "$(dirname "$0")/../rust-crdt_amd" || exit 2
mkdir -p build_stats
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -DMAP_STATS -I../include -Icsrc -x hip -c csrc/map.hip -o build_stats/map.hip.o || exit 1
objs=$(ls build/*.o | grep -v '/map.hip.o')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libcrdt_gpu_stats.so $objs build_stats/map.hip.o -ldl -Wl,-rpath,/opt/rocm/lib
