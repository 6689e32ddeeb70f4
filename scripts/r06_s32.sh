#!/bin/bash
# Round-6 session 32: Map merge_batch (8,192 pairs x 1,024 keys) with the states in contiguous device
# blocks against the torch allocator, interleaved on one box, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for v in contig torch; do
    f=--contig; [ $v = torch ] && f=
    timeout -k 10 300 python -u scripts/bench_merge_batch.py --only map $f > gpurun_out/r06_s32_${v}_$rep.log 2>&1 || exit $?
    echo "map_merge $v $rep $(grep -o '"kernel_ms_incl_deferred": [0-9.]*\|"frac_of_8TBs": [0-9.]*\|"parity": "[A-Za-z]*"' gpurun_out/r06_s32_${v}_$rep.log | tr '\n' ' ')"
  done
done
