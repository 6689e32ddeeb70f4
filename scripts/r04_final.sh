#!/bin/bash
# Round-4 closing check: every GPU test, smoke(), then the Map<K, Orswot> / counter Map benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r04c.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_r04c.log | head -20; tail -n 2 gpurun_out/pytest_gpu_r04c.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04c.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_r04c.log
bash scripts/gpu.sh run r04_map_orswot bash scripts/r04_mo_bench.sh
