#!/bin/bash
# Map<K, Orswot> adaptive chunk skip: its tests, then the A/B on both inputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_gpu_map_orswot.py > gpurun_out/pytest_r05_s5.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_r05_s5.log | head; tail -n 2 gpurun_out/pytest_r05_s5.log
[ $rc -ne 0 ] && exit $rc
bash scripts/r05_mo_ab.sh
