#!/bin/bash
# Round-6 session 24: the deep pass for long live Map-remove lists (Map<K, Orswot>, nested Map), with
# the deep / fold / apply tests of both types.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_map_orswot_deep.py tests/test_gpu_map_nested_deep.py tests/test_gpu_map_orswot.py tests/test_gpu_map_nested.py tests/test_gpu_vmap_merge.py tests/test_gpu_shard_abi.py -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/r06_s24_tests.log 2>&1
rc=$?; tail -n 20 gpurun_out/r06_s24_tests.log; exit $rc
