#!/bin/bash
# Round-5 step 1: the round's new / changed GPU tests, then bench.py with the new c3 / c4 blocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_gpu_map_nested.py tests/test_gpu_map_counter.py tests/test_gpu_map_orswot.py tests/test_gpu_shard_abi.py tests/test_gpu_dist_world2.py tests/test_gpu_bench_launch.py tests/test_gpu_lattice_multi.py > gpurun_out/pytest_r05a.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_r05a.log | head -30; grep -iE "RuntimeWarning|rccl" gpurun_out/pytest_r05a.log | head -5; tail -n 3 gpurun_out/pytest_r05a.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r05a.log 2>&1; rc2=$?
echo "bench rc=$rc2"; grep '^{' gpurun_out/bench_r05a.log | cut -c1-300; tail -n 5 gpurun_out/bench_r05a.log | cut -c1-300
exit $rc2
