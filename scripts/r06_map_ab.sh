#!/bin/bash
# Config-4 Map fold (RS path): A/B of map.hip build variants (CRDT_GPU_LIB), interleaved, twice each;
# bench_map.py checks parity on 8 sampled keys every run.
#   base  : the committed build
#   ws8   : -DMAP_RS_WS8=1 (step stride 8 mod 32 words: conflict-free reloads)
#   nt    : -DMAP_RS_NT=1 (non-temporal LDS-DMA)
#   wsnt  : both
# (round 6 earlier: tbinc -DMAP_TB_INC=1 2.27-2.28, vanm -DMAP_VAN_MASK=1 2.41, both 2.34 vs base 2.235 ms)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for v in base ${AB_VARIANTS:-ws8 nt wsnt}; do
    lib=rust-crdt_amd/libcrdt_gpu.so; [ $v != base ] && lib=rust-crdt_amd/libcrdt_gpu_$v.so
    CRDT_GPU_LIB=$PWD/$lib timeout -k 10 200 python -u scripts/bench_map.py --steps 10 --cpu-replicas 16 > gpurun_out/r06_map_${AB_TAG:-ab2}_${v}_$rep.log 2>&1 || exit $?
    echo "$v $rep $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/r06_map_${AB_TAG:-ab2}_${v}_$rep.log) $(grep -o '"parity": "[A-Za-z]*"' gpurun_out/r06_map_${AB_TAG:-ab2}_${v}_$rep.log)"
  done
done
