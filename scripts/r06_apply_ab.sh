#!/bin/bash
# Value-Map apply A/B on one box: the current library against variants (AB_VARIANTS, default r5ap =
# libcrdt_gpu_r5ap.so, the round-5 apply kernels linked with everything else current),
# bench_vmap_ops at Dcap 16 (the round-5 limit), interleaved, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for v in cur ${AB_VARIANTS:-r5ap}; do
    lib=rust-crdt_amd/libcrdt_gpu.so; [ $v != cur ] && lib=rust-crdt_amd/libcrdt_gpu_$v.so
    CRDT_GPU_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/bench_vmap_ops.py --dcap ${AB_DCAP:-16} > gpurun_out/r06_apply_ab_${v}_$rep.log 2>&1 || exit $?
    echo "$v $rep $(grep -o '"op": "map_[a-z]*_apply_batch[^"]*", "states": [0-9]*, "ops_per_state": [0-9]*, "actors": [0-9]*, "kernel_us": [0-9.]*' gpurun_out/r06_apply_ab_${v}_$rep.log | sed 's/"states.*kernel_us"//' | tr '\n' ' ')"
  done
done
