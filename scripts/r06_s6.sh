#!/bin/bash
# Round-6 session 6: value-Map apply with deferred slots past the 16 held in LDS (in place in the
# caller's slot arrays): the apply GPU tests, then bench_vmap_ops at Dcap 64 (status 0, parity over
# every sampled state) and at the round-5 Dcap 16 (timing unchanged by the two-tier list).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map_counter_apply.py tests/test_gpu_map_orswot_apply.py tests/test_gpu_map_nested_apply.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_s6_apply.log 2>&1
rc=$?; tail -n 3 gpurun_out/r06_s6_apply.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s6_vmap64.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_s6_vmap64.log | cut -c1-330
timeout -k 10 400 python -u scripts/bench_vmap_ops.py --dcap 16 > gpurun_out/r06_s6_vmap16.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_s6_vmap16.log | cut -c1-200
echo "session 6 done"
