#!/bin/bash
# Map forget: with vs without bench_forget.py's Orswot workload first in the same process.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --orswot-first --reset copy --tag o$i > gpurun_out/spread_ofirst_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --orswot-first --tag os$i > gpurun_out/spread_ofirst_synth_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --reset copy --tag n$i > gpurun_out/spread_nofirst_$i.log 2>&1 || exit $?
  grep -h map_forget gpurun_out/spread_ofirst_$i.log gpurun_out/spread_ofirst_synth_$i.log gpurun_out/spread_nofirst_$i.log | cut -c1-260
done
