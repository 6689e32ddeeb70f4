#!/bin/bash
# Counter-Map whole-chunk skip: parity in every mode, then the config-4-shape bench A/B (mccs=1 / 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_gpu_map_counter.py tests/test_gpu_map_nested.py "tests/test_gpu_host_mem.py::test_map_counter_host_lub_many" "tests/test_gpu_host_mem.py::test_map_orswot_host_lub_many" "tests/test_gpu_host_mem.py::test_map_nested_host_lub_many" > gpurun_out/pytest_r05_mc.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_r05_mc.log | head; tail -n 3 gpurun_out/pytest_r05_mc.log
[ $rc -ne 0 ] && exit $rc
for t in "" "mccs=0" ""; do
  CRDT_TUNE=$t timeout -k 10 300 python -u scripts/bench_map_counter.py > gpurun_out/r05_mc_bench_$t.log 2>&1 || exit $?
  echo "tune=$t"; grep '^{' gpurun_out/r05_mc_bench_$t.log | cut -c1-400
done
