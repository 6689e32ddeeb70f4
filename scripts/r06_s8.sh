#!/bin/bash
# Round-6 session 8: value-typed Map merge_batch (counter / orswot / nested, over the fold kernels)
# against the oracle's Map.merge; bench_vmap_ops again (counter apply timing after the slot zeroing).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_vmap_merge.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_s8_tests.log 2>&1
rc=$?; tail -n 30 gpurun_out/r06_s8_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s8_vmap64.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_s8_vmap64.log | cut -c1-200
echo "session 8 done"
