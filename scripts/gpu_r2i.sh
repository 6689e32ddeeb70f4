#!/bin/bash
# Map forget: does the size of the allocation the buffers live in set the speed?
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for c in 0 13 16 32 64; do
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --carve-gib $c --tag g$c > gpurun_out/spread_carve_$c.log 2>&1 || exit $?
  grep -h map_forget gpurun_out/spread_carve_$c.log | cut -c1-230
done
timeout -k 10 200 python -u scripts/bench_forget_spread.py --slab --tag slab > gpurun_out/spread_carve_slab.log 2>&1 || exit $?
grep -h map_forget gpurun_out/spread_carve_slab.log | cut -c1-230
