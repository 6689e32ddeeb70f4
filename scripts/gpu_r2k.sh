#!/bin/bash
# Map forget spread, decisive runs: bench_forget.py with and without its Orswot part (buffer
# offsets printed), and the spread script with the state buffers at chosen offsets of one 32 GiB
# allocation.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/bench_forget.py > gpurun_out/fk_full.log 2>&1 || exit $?
FORGET_MAP_ONLY=1 timeout -k 10 200 python -u scripts/bench_forget.py > gpurun_out/fk_maponly.log 2>&1 || exit $?
grep -h map_forget gpurun_out/fk_full.log gpurun_out/fk_maponly.log | cut -c1-400
for o in 0 4 8 12.25 16.25; do
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --carve-gib 32 --offset-gib $o --tag off$o > gpurun_out/fk_off$o.log 2>&1 || exit $?
  grep -h map_forget gpurun_out/fk_off$o.log | cut -c1-250
done
