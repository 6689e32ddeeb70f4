#!/bin/bash
# NQ=2 Map fold + counter chunk-skip tests, the full-size configs, then the r05b profile passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_gpu_map.py tests/test_gpu_map_counter.py tests/test_gpu_map_orswot.py tests/test_gpu_fullsize.py tests/test_gpu_kat.py > gpurun_out/pytest_r05_s4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_r05_s4.log | head; tail -n 2 gpurun_out/pytest_r05_s4.log
[ $rc -ne 0 ] && exit $rc
bash profiles/collect.sh r05b
timeout -k 10 300 python -u scripts/bench_map_orswot.py > gpurun_out/r05_mo_bench.log 2>&1 || exit $?
CRDT_TUNE=mocs=0 timeout -k 10 300 python -u scripts/bench_map_orswot.py > gpurun_out/r05_mo_bench_off.log 2>&1 || exit $?
grep '^{' gpurun_out/r05_mo_bench.log gpurun_out/r05_mo_bench_off.log | cut -c1-300
