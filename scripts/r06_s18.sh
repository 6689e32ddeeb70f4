#!/bin/bash
# Round-6 session 18: the nested Map fold with inner key sets past 64 (K2 <= 256): the nested fold
# tests (op-replay folds at K2 = 100 / 130 / 256, the TMap laws over the whole u8 domain), the value-
# Map merge / wire / apply tests at their round-5 shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_map_nested.py tests/test_gpu_map_nested_apply.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/r06_s18_tests.log 2>&1
rc=$?; tail -n 25 gpurun_out/r06_s18_tests.log; exit $rc
