#!/bin/bash
# Map merge_batch register kernel: parity (both kernels) and throughput A/B.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_merge_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_merge_batch.log 2>&1
rc=$?; tail -n 15 gpurun_out/pytest_merge_batch.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_merge_batch.py > gpurun_out/bench_merge_batch.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_merge_batch.log
CRDT_TUNE=mpreg=0 timeout -k 10 400 python -u scripts/bench_merge_batch.py > gpurun_out/bench_merge_batch_generic.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_merge_batch_generic.log
