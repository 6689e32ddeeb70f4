#!/bin/bash
# Round-6 session 23: MAP_RS_LATE (the slot-read wait moved into the spread DMA hook, pieces one
# element later): the Map fold tests, config-4 full-size parity, then an interleaved A/B against
# -DMAP_RS_LATE=0 (early) with bench_map.py, twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s23_tests.log 2>&1
rc=$?; tail -n 4 gpurun_out/r06_s23_tests.log; [ $rc -eq 0 ] || exit $rc
AB_TAG=late AB_VARIANTS="early" bash scripts/r06_map_ab.sh
