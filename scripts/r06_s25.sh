#!/bin/bash
# Round-6 session 25: nested Map value slots past 8 (Vs, up to 64): the deep tests and every nested /
# value-Map GPU test, the host-memory tests; then the nested fold bench and the value-Map ops bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_map_nested_deep.py tests/test_gpu_map_nested.py tests/test_gpu_map_nested_apply.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py tests/test_gpu_host_mem.py tests/test_gpu_map_orswot_deep.py tests/test_abi.py tests/test_gpu_shard_abi.py -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/r06_s25_tests.log 2>&1
rc=$?; tail -n 30 gpurun_out/r06_s25_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_map_nested.py > gpurun_out/r06_s25_nested_bench.log 2>&1
rc=$?; tail -n 3 gpurun_out/r06_s25_nested_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s25_vmap_ops.log 2>&1
rc=$?; tail -n 8 gpurun_out/r06_s25_vmap_ops.log; exit $rc
