#!/bin/bash
# Run a subset of the GPU tests: bash scripts/gpu_tests.sh tests/test_x.py [more pytest args]
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 40 gpurun_out/pytest_sel.log
exit $rc
