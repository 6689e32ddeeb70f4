#!/bin/bash
# Round-6 session 30: the map_fold timer without the chunk-max kernel: the Map tests, then the default
# bench (every block, parity + CPU legs) and the rocprofv3 evidence of the same build (collect r06l).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s30_tests.log 2>&1 || exit $?
tail -n 1 gpurun_out/r06_s30_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r06l.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_r06l.log | cut -c1-200
bash profiles/collect.sh r06l
