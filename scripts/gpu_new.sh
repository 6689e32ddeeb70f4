cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_forget_states.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/new_tests.log 2>&1; rc=$?
tail -30 gpurun_out/new_tests.log
exit $rc
