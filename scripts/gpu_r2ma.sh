#!/bin/bash
# Map / Orswot apply with deferred slots spilling to HBM: parity + apply benches
set -o pipefail
mkdir -p gpu_out_tmp gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_map_apply.py tests/test_gpu_orswot_apply.py > gpurun_out/r2ma_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_map_apply.py > gpurun_out/r2ma_bench_map.log 2>&1 &&
timeout -k 10 200 python -u scripts/bench_orswot_apply.py > gpurun_out/r2ma_bench_orswot.log 2>&1
rc=$?
tail -3 gpurun_out/r2ma_tests.log; cat gpurun_out/r2ma_bench_map.log gpurun_out/r2ma_bench_orswot.log 2>/dev/null | tail -20
exit $rc
