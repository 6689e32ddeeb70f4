#!/bin/bash
# Config-3 Orswot join: the ballot-vote build (libcrdt_gpu_vb.so) against the default, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base vb; do
    lib=rust-crdt_amd/libcrdt_gpu.so; [ $v != base ] && lib=rust-crdt_amd/libcrdt_gpu_$v.so
    CRDT_GPU_LIB=$PWD/$lib timeout -k 10 200 python -u scripts/bench_orswot.py --steps 8 > gpurun_out/r05_or_ab_${v}_$rep.log 2>&1 || exit $?
    echo "$v $rep $(grep -o '"join_ms": [0-9.]*' gpurun_out/r05_or_ab_${v}_$rep.log) $(grep -o '"parity": "[A-Za-z]*"' gpurun_out/r05_or_ab_${v}_$rep.log)"
  done
done
