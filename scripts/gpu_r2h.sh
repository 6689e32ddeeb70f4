#!/bin/bash
# merge_batch with the 2R+1W calibration line; Map forget spread: bench_forget.py and the spread
# script with copy-reset vs regenerate-reset, 3 processes each.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_merge_batch.py > gpurun_out/bench_merge_batch.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_merge_batch.log | cut -c1-250
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/bench_forget.py > gpurun_out/forget_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --reset copy --tag c$i > gpurun_out/spread_copy_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --reset synth --tag s$i > gpurun_out/spread_synth_$i.log 2>&1 || exit $?
  grep -h map_forget gpurun_out/forget_$i.log gpurun_out/spread_copy_$i.log gpurun_out/spread_synth_$i.log | cut -c1-200
done
