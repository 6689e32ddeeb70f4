#!/bin/bash
# Round-4 last check on the final build: every GPU test, smoke(), bench.py at N=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r04d.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_r04d.log | head -20; tail -n 2 gpurun_out/pytest_gpu_r04d.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04d.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_r04d.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r04d.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_r04d.log | cut -c1-300
