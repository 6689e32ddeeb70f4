#!/bin/bash
# Round-6 session 7: non-temporal RS/ST LDS-DMA as the default (config-4 map fold) and zeroed vacated
# deferred slots in the value-Map applies: the map fold + apply GPU tests, bench_vmap_ops at Dcap 64
# (wire round trips equal now that vacated slots are zero), bench_map.py config 4 twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map.py tests/test_gpu_map_counter_apply.py tests/test_gpu_map_orswot_apply.py tests/test_gpu_map_nested_apply.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_s7_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r06_s7_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s7_vmap64.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_s7_vmap64.log | cut -c1-330
for rep in 1 2; do
  timeout -k 10 200 python -u scripts/bench_map.py --steps 10 --cpu-replicas 16 > gpurun_out/r06_s7_map_$rep.log 2>&1 || exit $?
  echo "map $rep $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/r06_s7_map_$rep.log) $(grep -o '"parity": "[A-Za-z]*"' gpurun_out/r06_s7_map_$rep.log)"
done
echo "session 7 done"
