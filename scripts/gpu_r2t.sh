#!/bin/bash
# Host-memory mode incl. the Orswot forms.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_mem.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_host_mem2.log 2>&1
rc=$?; tail -n 25 gpurun_out/pytest_host_mem2.log; exit $rc
