#!/bin/bash
# Round-6 session 19: nested apply / forget / merge_batch / wire with inner key sets past 64 (K2 <= 256,
# K2w mask words), then the value-Map ops bench (nested apply at K2 = 8 must stay where it was).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_map_nested_apply.py tests/test_gpu_map_nested.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/r06_s19_tests.log 2>&1
rc=$?; tail -n 25 gpurun_out/r06_s19_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s19_vmap_ops.log 2>&1
rc=$?; tail -n 12 gpurun_out/r06_s19_vmap_ops.log; exit $rc
