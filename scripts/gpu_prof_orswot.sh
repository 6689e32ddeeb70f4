#!/bin/bash
# Config-3 Orswot join on the GPU box: a tuning sweep (HIP events, parity each run), then the
# rocprofv3 kernel trace and the FETCH_SIZE / WRITE_SIZE passes of the chosen geometry.
#   bash scripts/gpu_prof_orswot.sh <tag> "<tune for the profile>" "<sweep tunes...>"
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
tag=${1:-r02_orswot_c3}
ptune=${2:-}
sweep=${3:-}
if [ -n "$sweep" ]; then
  timeout -k 10 400 python -u scripts/bench_orswot.py --steps 5 --tune $sweep > gpurun_out/sweep_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/sweep_$tag.log
fi
if [ -n "$ptune" ]; then B="scripts/bench_orswot.py --steps 5 --tune $ptune"; else B="scripts/bench_orswot.py --steps 5"; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 $B > gpurun_out/prof_$tag.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_$tag.log
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- python3 $B > gpurun_out/pmc_fetch_$tag.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$tag -o run -- python3 $B > gpurun_out/pmc_write_$tag.log 2>&1 || exit $?
# algorithmic bytes per join launch at config 3: 8*M*A + 8*A per replica, plus the output
python3 scripts/prof_summary.py $tag orswot_join_kernel $((65536 * (4096 * 64 * 8 + 64 * 8) + 4096 * 64 * 8 + 64 * 8))
