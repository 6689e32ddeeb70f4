cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for h in 4 1 0; do
  echo "== hot=$h"
  CRDT_TUNE=hot=$h timeout -k 10 200 python -u -m pytest tests/test_gpu_orswot_apply.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hot_$h.log 2>&1 || { tail -30 gpurun_out/hot_$h.log; exit 1; }
  tail -1 gpurun_out/hot_$h.log
done
for h in 4 2 8 16; do
  echo "== bench hot=$h"
  CRDT_TUNE=hot=$h timeout -k 10 200 python -u scripts/bench_orswot_apply.py > gpurun_out/bhot_$h.log 2>&1 || exit $?
  grep '^{' gpurun_out/bhot_$h.log | cut -c1-330
done
