#!/bin/bash
# Round-6 session 2: the SP path (two waves per key) of map_fold_kernel — parity first (every staging
# mode of test_gpu_map.py incl. msp=1, then config 4 at full size with both forms compared), then an
# A/B of config 4 (scripts/bench_map.py, HIP events, parity on 8 sampled keys) msp=0 vs msp=1, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_s2_map.log 2>&1
rc=$?; tail -n 5 gpurun_out/r06_s2_map.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k config4 --timeout 280 --timeout-method thread > gpurun_out/r06_s2_full.log 2>&1
rc=$?; tail -n 5 gpurun_out/r06_s2_full.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for t in msp=0 msp=1; do
    echo "== $t (run $i)" >> gpurun_out/r06_s2_ab.log
    CRDT_TUNE=$t timeout -k 10 200 python -u scripts/bench_map.py --steps 10 --cpu-replicas 16 >> gpurun_out/r06_s2_ab.log 2>&1 || exit $?
  done
done
grep -E "^==|kernel_ms|parity" gpurun_out/r06_s2_ab.log | cut -c1-300
echo "session 2 done"
