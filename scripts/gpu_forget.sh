cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_forget_states.py -x -v --timeout 120 --timeout-method thread > gpurun_out/forget_tests.log 2>&1; rc=$?
tail -12 gpurun_out/forget_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_forget.py > gpurun_out/bench_forget.log 2>&1 || exit $?
CRDT_TUNE=mfv2=0 timeout -k 10 300 python -u scripts/bench_forget.py > gpurun_out/bench_forget_novec.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_forget.log gpurun_out/bench_forget_novec.log
