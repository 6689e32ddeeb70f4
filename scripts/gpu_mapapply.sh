cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_map_apply.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mapapply_tests.log 2>&1; rc=$?
tail -30 gpurun_out/mapapply_tests.log
exit $rc
