#!/bin/bash
# Round-6: Map<K, GCounter / PNCounter> fold with the step-image LDS-DMA non-temporal (MC_AUX=2) vs
# the default policy, bench_map_counter.py, interleaved, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for v in base mcnt; do
    lib=rust-crdt_amd/libcrdt_gpu.so; [ $v != base ] && lib=rust-crdt_amd/libcrdt_gpu_$v.so
    CRDT_GPU_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/bench_map_counter.py > gpurun_out/r06_mc_ab_${v}_$rep.log 2>&1 || exit $?
    echo "$v $rep $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/r06_mc_ab_${v}_$rep.log | tr '\n' ' ') $(grep -o '"parity": "[A-Za-z]*"' gpurun_out/r06_mc_ab_${v}_$rep.log | tr '\n' ' ')"
  done
done
