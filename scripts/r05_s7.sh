#!/bin/bash
# Map<K, Orswot> wide kernel (A > 64 / M > 32 / mowide=1) and host-memory mode tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_gpu_map_orswot.py tests/test_gpu_host_mem.py > gpurun_out/pytest_r05_s7.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_r05_s7.log | head; tail -n 3 gpurun_out/pytest_r05_s7.log
exit $rc
