#!/bin/bash
# Orswot / Map egress with batched rows and ballot counts: parity (wire tests) and throughput.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_wire_egress.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_wire_egress.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/bench_wire.py --skip gcounter,pncounter > gpurun_out/bench_wire_egress.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_wire_egress.log | cut -c1-600
