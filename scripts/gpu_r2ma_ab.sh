#!/bin/bash
# Apply kernels: parity, then A/B of the Map and Orswot apply benches, a previous library (ab/)
# vs the working tree's, alternating
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_map_apply.py tests/test_gpu_orswot_apply.py > gpurun_out/r2ma_tests.log 2>&1 || { tail -30 gpurun_out/r2ma_tests.log; exit 1; }
tail -2 gpurun_out/r2ma_tests.log
out=gpurun_out/r2ma_ab.log; : > $out
for i in 1 2; do
  for b in bench_map_apply bench_orswot_apply; do
    echo "== prev $b" >> $out
    CRDT_GPU_LIB=$PWD/ab/libcrdt_gpu_prev.so timeout -k 10 200 python -u scripts/$b.py >> $out 2>&1 || exit 1
    echo "== new $b" >> $out
    timeout -k 10 200 python -u scripts/$b.py >> $out 2>&1 || exit 1
  done
done
grep -o '== .*\|kernel_us": [0-9.]*\|"parity": "[a-z]*"' $out
