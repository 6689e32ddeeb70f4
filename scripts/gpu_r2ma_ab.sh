#!/bin/bash
# Map apply deferred spill: parity, then A/B of the apply bench, HEAD library (ab/) vs the working tree's
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_map_apply.py tests/test_gpu_orswot_apply.py > gpurun_out/r2ma_tests.log 2>&1 || { tail -30 gpurun_out/r2ma_tests.log; exit 1; }
tail -2 gpurun_out/r2ma_tests.log
out=gpurun_out/r2ma_ab.log; : > $out
for i in 1 2; do
  echo "== prev" >> $out
  CRDT_GPU_LIB=$PWD/ab/libcrdt_gpu_prev.so timeout -k 10 200 python -u scripts/bench_map_apply.py >> $out 2>&1 || exit 1
  echo "== new" >> $out
  timeout -k 10 200 python -u scripts/bench_map_apply.py >> $out 2>&1 || exit 1
done
grep -o '== .*\|kernel_us": [0-9.]*' $out
