#!/bin/bash
# Counter-Map apply: op headers staged in LDS per 64-op batch (CRDT_MCA_HDR=2, the variant build
# scripts/build_variant.sh mcahdr2 map_counter_apply.hip -DCRDT_MCA_HDR=2) against the default
# (one global read per field per op): the counter-Map apply parity tests on the variant, then
# bench_vmap_ops.py alternated between the builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
V=$PWD/rust-crdt_amd/libcrdt_gpu_mcahdr2.so
CRDT_GPU_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_map_counter_apply.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05_mcahdr2_tests.log 2>&1 || { tail -n 30 gpurun_out/r05_mcahdr2_tests.log; exit 1; }
echo "tests: $(tail -n 1 gpurun_out/r05_mcahdr2_tests.log)"
for rep in 1 2; do
  for v in hdr2 hdr0; do
    if [ $v = hdr2 ]; then export CRDT_GPU_LIB=$V; else unset CRDT_GPU_LIB; fi
    timeout -k 10 300 python -u scripts/bench_vmap_ops.py --reps 5 > gpurun_out/r05_mcahdr2_${v}_$rep.log 2>&1 || exit $?
    echo "== $v rep $rep"; grep -o '"op": "map_[a-z_]*apply[^"]*"\|"kernel_us": [0-9.]*\|"parity": "[a-z]*"' gpurun_out/r05_mcahdr2_${v}_$rep.log | paste - - - | head -1
  done
done
