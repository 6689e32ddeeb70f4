#!/bin/bash
# Round-6 checkpoint: the full `-m gpu` suite, smoke(), bench.py at N = 1 (every block), then
# bench.py's N > 1 code path at world 2 on this one GPU (gloo + the C ABI's caller-collectives seam).
set -o pipefail
tag=${1:-r06c}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$tag.log | head; tail -n 2 gpurun_out/pytest_$tag.log
grep -c "RuntimeWarning" gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_$tag.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_$tag.log | cut -c1-400
[ "${CKPT_WORLD2:-1}" = 1 ] || exit 0
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --exchange cabi-ops --steps 5 --warmup 1 \
  --no-cpu-baseline > gpurun_out/bench_world2_$tag.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_world2_$tag.log | cut -c1-400
