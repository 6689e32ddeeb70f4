cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_abi.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/shard_tests.log 2>&1; rc=$?
tail -40 gpurun_out/shard_tests.log
exit $rc
