#!/bin/bash
# Orswot apply with LDS-staged Rm clock rows: tests, then the A/B (default vs oastg=0), 3 reps interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_gpu_orswot_apply.py > gpurun_out/pytest_r05_s9.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_r05_s9.log | head; tail -n 2 gpurun_out/pytest_r05_s9.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for t in "" "oastg=0"; do
    timeout -k 10 200 python -u scripts/bench_orswot_apply.py --tune "$t" > gpurun_out/r05_oastg_${rep}_$t.log 2>&1 || exit $?
    echo "tune=[$t] $rep $(grep -o '"kernel_ms": [0-9.]*\|"kernel_us": [0-9.]*\|"parity": "[A-Za-z]*"' gpurun_out/r05_oastg_${rep}_$t.log | tr '\n' ' ')"
  done
done
