#!/bin/bash
# Round-6 session 15: the value-typed Maps' merge_batch through the C ABI (csrc/vmap_merge.hip).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_vmap_merge.py tests/test_gpu_map_counter_apply.py tests/test_gpu_wire_vmap.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_s15_tests.log 2>&1
rc=$?; tail -n 30 gpurun_out/r06_s15_tests.log; exit $rc
