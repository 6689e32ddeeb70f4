#!/bin/bash
# The one GPU-box runner (replaces the per-session gpu_*.sh scripts).  Run through gpurun from the
# repository root, e.g.  gpurun -- 'bash scripts/gpu.sh tests tests/test_gpu_map.py'
#   tests <pytest args>          GPU tests (-m gpu), log gpurun_out/pytest_<n>.log
#   round <tag>                  the round checkpoint: every GPU test, smoke(), bench.py, then the
#                                rocprofv3 evidence of the bench's dominant kernel (profiles/collect.sh)
#   run <tag> <cmd...>           any command (a scripts/bench_*.py), output gpurun_out/<tag>.log
#   trace <tag> <cmd...>         rocprofv3 kernel trace + stats of a command -> gpurun_out/prof_<tag>/
#   pmc <tag> <ctr,..> <cmd...>  one rocprofv3 counter pass (one pass per call: the box refuses more
#                                counters than a block collects at once) -> gpurun_out/pmc_<tag>/
# Every GPU step runs under its own timeout and the steps stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
mode=$1; shift
case "$mode" in
  tests)
    n=$(date +%s)
    timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_$n.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_$n.log; exit $rc ;;
  testsall)  # every test runs (no -x); rc 1 = some failed, any other nonzero rc = stop
    n=$(date +%s)
    timeout -k 10 1000 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_$n.log 2>&1
    rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$n.log | head -40; tail -n 3 gpurun_out/pytest_$n.log; exit $rc ;;
  round)
    tag=${1:-r03}
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$tag.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_gpu_$tag.log; [ $rc -ne 0 ] && exit $rc
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
    tail -n 1 gpurun_out/smoke_$tag.log
    timeout -k 10 300 python -u bench.py > gpurun_out/bench_$tag.log 2>&1 || exit $?
    grep '^{' gpurun_out/bench_$tag.log | cut -c1-400
    bash profiles/collect.sh "$tag" ;;
  run)
    tag=$1; shift
    timeout -k 10 600 "$@" > gpurun_out/$tag.log 2>&1; rc=$?
    tail -n 20 gpurun_out/$tag.log; exit $rc ;;
  trace)
    tag=$1; shift
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- "$@" > gpurun_out/prof_$tag.log 2>&1; rc=$?
    tail -n 5 gpurun_out/prof_$tag.log; exit $rc ;;
  pmc)
    tag=$1; ctr=$2; shift 2
    timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d gpurun_out/pmc_$tag -o run -- "$@" > gpurun_out/pmc_$tag.log 2>&1; rc=$?
    tail -n 5 gpurun_out/pmc_$tag.log; exit $rc ;;
  *)
    echo "usage: scripts/gpu.sh tests|round|run|trace|pmc ..." >&2; exit 2 ;;
esac
