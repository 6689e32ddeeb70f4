#!/bin/bash
# Nested-Map apply with the header batch: 5 waves per SIMD (CRDT_MNA_WPE=5, variant) vs the compiler default 4;
# parity tests on the variant, then bench_vmap_ops.py alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in mnaw5; do
  CRDT_GPU_LIB=$PWD/rust-crdt_amd/libcrdt_gpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_map_nested_apply.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r05_mna_${v}_tests.log 2>&1 || { tail -n 30 gpurun_out/r05_mna_${v}_tests.log; exit 1; }
  echo "$v tests: $(tail -n 1 gpurun_out/r05_mna_${v}_tests.log)"
done
for rep in 1 2; do
  for v in def mnaw5; do
    if [ $v = def ]; then unset CRDT_GPU_LIB; else export CRDT_GPU_LIB=$PWD/rust-crdt_amd/libcrdt_gpu_$v.so; fi
    timeout -k 10 300 python -u scripts/bench_vmap_ops.py --reps 5 > gpurun_out/r05_mna_${v}_$rep.log 2>&1 || exit $?
    echo "== $v rep $rep"; grep -o '"op": "map_[a-z_]*apply[^"]*"\|"kernel_us": [0-9.]*\|"parity": "[a-z]*"' gpurun_out/r05_mna_${v}_$rep.log | paste - - - | sed -n 3p
  done
done
