#!/bin/bash
# Map<K, Orswot> fold: chunk skip (mocs=1) vs the register ring (mocs=0, the default) vs the ring at
# depth 4 (libcrdt_gpu_d4.so, occupancy 2), on the random and the causal (config-4 generator) inputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for inp in ${INPUTS:-random causal}; do
  for v in cs ring d4; do
    lib=rust-crdt_amd/libcrdt_gpu.so; tune="mocs=1"
    [ $v = ring ] && tune="mocs=0"
    [ $v = d4 ] && { lib=rust-crdt_amd/libcrdt_gpu_d4.so; tune="mocs=0"; }
    CRDT_TUNE=$tune CRDT_GPU_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/bench_map_orswot.py --input $inp > gpurun_out/r05_mo_ab_${inp}_$v.log 2>&1 || exit $?
    echo "$inp $v $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/r05_mo_ab_${inp}_$v.log) $(grep -o '"parity": "[A-Za-z]*"' gpurun_out/r05_mo_ab_${inp}_$v.log)"
  done
done
