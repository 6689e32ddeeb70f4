cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_map_apply.py tests/test_gpu_orswot_apply.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mapapply_tests.log 2>&1; rc=$?
tail -12 gpurun_out/mapapply_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_map_apply.py > gpurun_out/bench_mapapply.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_mapapply.log
timeout -k 10 300 python -u scripts/bench_orswot_apply.py > gpurun_out/bench_apply.log 2>&1 || exit $?
grep "^{" gpurun_out/bench_apply.log
