#!/bin/bash
# Round-6 session 13: (a) config-4 map fold LDS-DMA policy A/B (aux 2 = nt default, 16 = sc1, 18 = sc1 nt,
# 3 = sc0 nt); (b) Map<K, Orswot> fold at config-4 scale, causal input: level 1 of a replica split
# (the replicas cut into P groups) at ring depth 8 (default) / 4 / 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
AB_TAG=ab3 AB_VARIANTS="aux16 aux18 aux3" bash scripts/r06_map_ab.sh || exit $?
for v in base mod4 mod2; do
  lib=rust-crdt_amd/libcrdt_gpu.so; [ $v != base ] && lib=rust-crdt_amd/libcrdt_gpu_$v.so
  for P in 2 4 8; do
    CRDT_GPU_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/bench_map_orswot.py --input causal --split-probe $P --steps 3 > gpurun_out/r06_mosplit_${v}_$P.log 2>&1 || exit $?
    echo "$v P=$P $(grep -o '"level1_kernel_ms": [0-9.]*, "whole_kernel_ms": [0-9.]*' gpurun_out/r06_mosplit_${v}_$P.log) $(grep -o '"parity": "[A-Za-z]*"' gpurun_out/r06_mosplit_${v}_$P.log)"
  done
done
echo "session 13 done"
