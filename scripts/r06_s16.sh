#!/bin/bash
# Round-6 session 16: the nested Map fold at A <= 256 (NVc clocks, APL 1 / 2 / 4): the nested GPU tests
# (TMap laws with up to 256 actors, op-replay folds at A = 100 / 200 / 256), the value-Map merge tests,
# then bench_map_nested.py (the APL = 1 instance's speed against round 5's 30.0 ms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_map_nested.py tests/test_gpu_map_nested_apply.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s16_tests.log 2>&1
rc=$?; tail -n 25 gpurun_out/r06_s16_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_map_nested.py > gpurun_out/r06_s16_nested.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_s16_nested.log | cut -c1-400
echo "session 16 done"
