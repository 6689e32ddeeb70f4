#!/bin/bash
# Map fold threshold scan (mscan3=1, default) vs the round-1 scan: parity + time A/B + full-size config 4 test.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_map.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_map_scan3.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_scan3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k map --timeout 280 --timeout-method thread > gpurun_out/pytest_map_full_scan3.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_full_scan3.log; [ $rc -ne 0 ] && exit $rc
for m in 1 0 1 0; do
  CRDT_TUNE=mscan3=$m timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 10 > gpurun_out/bench_map_scan3_$m.log 2>&1 || exit $?
  grep -h kernel_ms gpurun_out/bench_map_scan3_$m.log | cut -c150-330
done
