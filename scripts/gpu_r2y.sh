#!/bin/bash
# Map fold RS path with the scan operands held in registers (default) vs read from LDS per chunk (previous build): parity, time A/B, phase cycles.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_map.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_map_rsr.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_rsr.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k map --timeout 280 --timeout-method thread > gpurun_out/pytest_map_full_rsr.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_full_rsr.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in rsr prev; do
    case $v in
      rsr) env="" ;; prev) env="CRDT_GPU_LIB=$PWD/rust-crdt_amd/ab/libcrdt_gpu_prev.so" ;;
    esac
    env $env timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 10 > gpurun_out/bench_map_$v.log 2>&1 || exit $?
    echo "$v $(grep -h kernel_ms gpurun_out/bench_map_$v.log | cut -c150-260)"
  done
done
timeout -k 10 300 python -u scripts/bench_map.py --steps 5 > gpurun_out/bench_map_rsr_parity.log 2>&1 || exit $?
grep -h kernel_ms gpurun_out/bench_map_rsr_parity.log | cut -c1-400
CRDT_GPU_LIB=$PWD/rust-crdt_amd/ab/libcrdt_gpu_stats.so timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 1 > gpurun_out/stats_map_rsr.log 2>&1 || exit $?
grep -h "k=" gpurun_out/stats_map_rsr.log | tail -n 4
