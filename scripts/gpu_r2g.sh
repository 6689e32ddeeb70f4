#!/bin/bash
# Orswot merge_batch: parity at every row-block size, then throughput A/B over prows.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 64 256 128; do
  CRDT_TUNE=prows=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_merge_batch.py -x -q -k orswot --timeout 120 --timeout-method thread > gpurun_out/pytest_mb_prows$r.log 2>&1
  rc=$?; tail -n 2 gpurun_out/pytest_mb_prows$r.log; [ $rc -ne 0 ] && exit $rc
done
for r in 64 128 256; do
  CRDT_TUNE=prows=$r timeout -k 10 400 python -u scripts/bench_merge_batch.py --map-pairs 16 > gpurun_out/bench_mb_prows$r.log 2>&1 || exit $?
  grep -h orswot gpurun_out/bench_mb_prows$r.log | cut -c1-200
done
