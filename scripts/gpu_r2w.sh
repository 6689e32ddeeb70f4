#!/bin/bash
# Map fold register-staged whole-chunk skip (mrs=1, default) vs the LDS-DMA ring: parity, full-size config 4, time A/B, phase cycles.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_merge_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_map_rs.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_rs.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k map --timeout 280 --timeout-method thread > gpurun_out/pytest_map_full_rs.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_full_rs.log; [ $rc -ne 0 ] && exit $rc
for m in 1 0 1 0; do
  CRDT_TUNE=mrs=$m timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 10 > gpurun_out/bench_map_rs_$m.log 2>&1 || exit $?
  grep -h kernel_ms gpurun_out/bench_map_rs_$m.log | cut -c150-330
done
timeout -k 10 300 python -u scripts/bench_map.py --steps 5 > gpurun_out/bench_map_rs_parity.log 2>&1 || exit $?
grep -h kernel_ms gpurun_out/bench_map_rs_parity.log | cut -c1-400
for m in 1 0; do
  CRDT_GPU_LIB=$PWD/rust-crdt_amd/ab/libcrdt_gpu_stats.so CRDT_TUNE=mrs=$m timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 1 > gpurun_out/stats_map_rs_$m.log 2>&1 || exit $?
  grep -h "k=" gpurun_out/stats_map_rs_$m.log | tail -n 4
done
