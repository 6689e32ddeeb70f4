#!/bin/bash
# Round-6 session 17: the TMap merge laws with up to 256 actors (no skips expected).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map_nested.py -x -v -rs --timeout 300 --timeout-method thread -k "wide or op_replay" > gpurun_out/r06_s17_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/r06_s17_tests.log | tail -n 30; exit $rc
