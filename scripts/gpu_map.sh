#!/bin/bash
# Map fold on the GPU box: parity tests, then the config-4 bench (exact, then other slice counts).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_map.py -x -q --timeout 120 --timeout-method thread > gpurun_out/map_tests.log 2>&1
rc=$?; tail -3 gpurun_out/map_tests.log; [ $rc -ne 0 ] && exit $rc
n=0
for tune in ${TUNES:-default}; do
  n=$((n+1))
  [ "$tune" = default ] && tune=""
  CRDT_TUNE="$tune" timeout -k 10 240 python -u scripts/bench_map.py --cpu-replicas 64 ${BENCH_ARGS} > gpurun_out/bench_map_$n.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/bench_map_$n.log | grep '^{"workload\|parity'; [ $rc -ne 0 ] && [ $rc -ne 3 ] && exit $rc
done
echo "== all done"
