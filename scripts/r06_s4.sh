#!/bin/bash
# Round-6 session 4: the world-2 C-ABI tests (agreed-plan cache), config 4 at full size with both
# Map-fold forms compared, then the config-4 A/B msp=0 vs msp=1 (twice).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_world2.py -x -q --timeout 500 --timeout-method thread > gpurun_out/r06_s4_w2.log 2>&1
rc=$?; tail -n 3 gpurun_out/r06_s4_w2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k config4 --timeout 280 --timeout-method thread > gpurun_out/r06_s4_full.log 2>&1
rc=$?; tail -n 3 gpurun_out/r06_s4_full.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for t in msp=0 msp=1; do
    echo "== $t (run $i)" >> gpurun_out/r06_s4_ab.log
    CRDT_TUNE=$t timeout -k 10 200 python -u scripts/bench_map.py --steps 10 --cpu-replicas 16 >> gpurun_out/r06_s4_ab.log 2>&1 || exit $?
  done
done
grep -E "^==|kernel_ms|parity" gpurun_out/r06_s4_ab.log | cut -c1-260
echo "session 4 done"
