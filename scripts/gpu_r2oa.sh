#!/bin/bash
# Orswot apply with atomic-max adds: parity (all apply tests) and the bench (65,536 states x 64 ops).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_orswot_apply.py tests/test_gpu_kat.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_oapply_atomic.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_oapply_atomic.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_orswot_apply.py > gpurun_out/bench_oapply_atomic.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_oapply_atomic.log | cut -c1-500
