#!/bin/bash
# Round-6 session 20: Map<K, Orswot> past 16 nested deferred removes per key (Vd slots, ABI 8): the new
# deep tests, every Map<K, Orswot> / value-Map GPU test, the ABI tests; then the fold bench (default
# Vd = 16 must stay where it was) and the value-Map ops bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_map_orswot_deep.py tests/test_gpu_map_orswot.py tests/test_gpu_map_orswot_apply.py tests/test_gpu_map_value_forget.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py tests/test_gpu_host_mem.py tests/test_abi.py -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/r06_s20_tests.log 2>&1
rc=$?; tail -n 30 gpurun_out/r06_s20_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_map_orswot.py > gpurun_out/r06_s20_mo_bench.log 2>&1
rc=$?; tail -n 6 gpurun_out/r06_s20_mo_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s20_vmap_ops.log 2>&1
rc=$?; tail -n 8 gpurun_out/r06_s20_vmap_ops.log; exit $rc
