cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_forget_states.py -x -q --timeout 120 --timeout-method thread > gpurun_out/forget_tests.log 2>&1 || { tail -30 gpurun_out/forget_tests.log; exit 1; }
tail -2 gpurun_out/forget_tests.log
for b in 4; do
  echo "== rows_blocks_per_cu=$b"
  CRDT_TUNE=rbpc=$b timeout -k 10 200 python -u scripts/bench_forget.py > gpurun_out/forget_b$b.log 2>&1 || exit $?
  grep '^{' gpurun_out/forget_b$b.log | cut -c1-200
done
