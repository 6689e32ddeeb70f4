#!/bin/bash
# Round checkpoint on the GPU box: the whole -m gpu suite, smoke, the bench, and the rocprofv3
# evidence of the bench's dominant kernel (kernel trace + FETCH_SIZE + WRITE_SIZE passes).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
tag=${1:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_gpu_$tag.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_$tag.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_$tag.log
bash profiles/collect.sh $tag
