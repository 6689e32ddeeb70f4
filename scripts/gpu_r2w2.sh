#!/bin/bash
# Map wire ingest through the LDS frame window: parity (all wire tests) and throughput vs the direct kernel.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_map.py -x -q --timeout 200 --timeout-method thread -k "wire or direct or long_folds" > gpurun_out/pytest_wire_win.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_wire_win.log; [ $rc -ne 0 ] && exit $rc
for m in 1 0; do
  CRDT_TUNE=wwin=$m timeout -k 10 500 python -u scripts/bench_wire.py --skip gcounter,pncounter,orswot > gpurun_out/bench_wire_map_w$m.log 2>&1 || exit $?
  echo "wwin=$m $(grep '^{' gpurun_out/bench_wire_map_w$m.log | cut -c1-400)"
done
