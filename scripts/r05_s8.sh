#!/bin/bash
# Counter-Map chunk skip with LDS-staged chunks: tests, then the A/B against register-staged chunks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_gpu_map_counter.py > gpurun_out/pytest_r05_s8.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_r05_s8.log | head; tail -n 2 gpurun_out/pytest_r05_s8.log
[ $rc -ne 0 ] && exit $rc
for t in "" mccl=0 mccs=0; do
  echo "== CRDT_TUNE=$t"
  CRDT_TUNE=$t timeout -k 10 300 python -u scripts/bench_map_counter.py > gpurun_out/r05_mccl_$t.log 2>&1 || exit $?
  grep -o '"value": "[A-Za-z]*"\|"kernel_ms": [0-9.]*\|"frac_of_8TBs": [0-9.]*\|"parity": "[A-Za-z]*"' gpurun_out/r05_mccl_$t.log | paste - - - -
done
