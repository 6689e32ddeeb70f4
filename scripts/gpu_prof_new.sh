#!/bin/bash
# rocprofv3 kernel-trace + stats for the round's §8f kernels (Orswot / Map apply, whole-state
# forget), each bench under its own profiler run; then a FETCH_SIZE and a WRITE_SIZE pass over
# the forget bench (HBM traffic of the streaming kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_oapply -o run -- python3 scripts/bench_orswot_apply.py --reps 3 > gpurun_out/prof_oapply.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mapply -o run -- python3 scripts/bench_map_apply.py --reps 3 > gpurun_out/prof_mapply.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_forget -o run -- python3 scripts/bench_forget.py > gpurun_out/prof_forget.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_forget -o run -- python3 scripts/bench_forget.py > gpurun_out/pmc_fetch_forget.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_forget -o run -- python3 scripts/bench_forget.py > gpurun_out/pmc_write_forget.log 2>&1 || exit $?
echo "== all done"
