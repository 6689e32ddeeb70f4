#!/bin/bash
# Round-6 session 9: value-Map applies as two passes (LDS-only pass for every state, the in-place
# tier for states whose Map deferred list outgrows the 16 LDS slots): apply GPU tests, then
# bench_vmap_ops at Dcap 64 and 16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map_counter_apply.py tests/test_gpu_map_orswot_apply.py tests/test_gpu_map_nested_apply.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_s9_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/r06_s9_tests.log; [ $rc -ne 0 ] && exit $rc
for dc in 64 16; do
  timeout -k 10 400 python -u scripts/bench_vmap_ops.py --dcap $dc > gpurun_out/r06_s9_vmap$dc.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06_s9_vmap$dc.log | cut -c1-260
done
echo "session 9 done"
