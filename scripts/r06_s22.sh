#!/bin/bash
# Round-6 session 22: the nested Map past 16 inner deferred removes per key (Id slots, ABI 8): the new
# deep tests, every nested / value-Map GPU test, ABI and host-memory tests; then the nested fold bench
# (default Id = 16 must stay where it was) and the value-Map ops bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_map_nested_deep.py tests/test_gpu_map_nested.py tests/test_gpu_map_nested_apply.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py tests/test_gpu_host_mem.py tests/test_gpu_map_orswot_deep.py tests/test_abi.py -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/r06_s22_tests.log 2>&1
rc=$?; tail -n 30 gpurun_out/r06_s22_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_map_nested.py > gpurun_out/r06_s22_nested_bench.log 2>&1
rc=$?; tail -n 4 gpurun_out/r06_s22_nested_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s22_vmap_ops.log 2>&1
rc=$?; tail -n 8 gpurun_out/r06_s22_vmap_ops.log; exit $rc
