#!/bin/bash
# Round-6 session 10: value-Map applies with the pass-1 body slimmed (resume written at the end, a
# 32-bit resume offset, no peak tracking in pass 1): apply GPU tests, the A/B against the round-5
# kernels at Dcap 16, then Dcap 64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map_counter_apply.py tests/test_gpu_map_orswot_apply.py tests/test_gpu_map_nested_apply.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_s10_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r06_s10_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r06_apply_ab.sh || exit $?
timeout -k 10 400 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s10_vmap64.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_s10_vmap64.log | cut -c1-260
echo "session 10 done"
