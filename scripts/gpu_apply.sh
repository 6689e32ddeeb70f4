cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_orswot_apply.py -x -v --timeout 120 --timeout-method thread > gpurun_out/apply_tests.log 2>&1; rc=$?
tail -30 gpurun_out/apply_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_orswot_apply.py > gpurun_out/apply_bench.log 2>&1; rc=$?
tail -5 gpurun_out/apply_bench.log
exit $rc
