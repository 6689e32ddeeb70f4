#!/bin/bash
# Nested-Map apply: op headers batched into lanes (CRDT_MNA_HDR=1, the default build) against one
# global read per field per op (scripts/build_variant.sh mnahdr0 map_nested_apply.hip -DCRDT_MNA_HDR=0):
# the nested apply parity tests on the default build, then bench_vmap_ops.py alternated between the builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_map_nested_apply.py tests/test_gpu_map_nested.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05_mnahdr_tests.log 2>&1 || { tail -n 30 gpurun_out/r05_mnahdr_tests.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/r05_mnahdr_tests.log)"
for rep in 1 2; do
  for v in hdr1 hdr0; do
    if [ $v = hdr0 ]; then export CRDT_GPU_LIB=$PWD/rust-crdt_amd/libcrdt_gpu_mnahdr0.so; else unset CRDT_GPU_LIB; fi
    timeout -k 10 300 python -u scripts/bench_vmap_ops.py --reps 5 > gpurun_out/r05_mnahdr_${v}_$rep.log 2>&1 || exit $?
    echo "== $v rep $rep"; grep -o '"op": "map_counter_apply[^"]*"\|"op": "map_[a-z_]*apply[^"]*"\|"kernel_us": [0-9.]*\|"parity": "[a-z]*"' gpurun_out/r05_mnahdr_${v}_$rep.log | paste - - - | head -6
  done
done
