#!/bin/bash
# Map fold: non-temporal LDS-DMA step images (CRDT_TUNE=mnt=1) vs default: parity, time, FETCH_SIZE.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out/pmc_mnt && export TMPDIR=/tmp
CRDT_TUNE=mnt=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_map.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_map_mnt.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_mnt.log; [ $rc -ne 0 ] && exit $rc
for m in 0 1 0 1; do
  CRDT_TUNE=mnt=$m timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 10 > gpurun_out/bench_map_mnt$m.log 2>&1 || exit $?
  grep -h kernel_ms gpurun_out/bench_map_mnt$m.log | cut -c1-330
done
for m in 0 1; do
  CRDT_TUNE=mnt=$m timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-include-regex map_fold --output-format csv -d gpurun_out/pmc_mnt/m$m -o run -- python3 scripts/prof_map.py > gpurun_out/pmc_mnt/m$m.log 2>&1 || exit $?
  tail -1 gpurun_out/pmc_mnt/m$m.log
done
