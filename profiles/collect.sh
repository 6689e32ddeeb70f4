#!/bin/bash
# Collect the rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command     -> gpurun_out/prof_<tag>/
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2)
# then summarises them into profiles/<tag>_*.csv / .json (scripts/summarize_prof.py).
tag=${1:-r02}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 $B > gpurun_out/prof_$tag.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- python3 $B > gpurun_out/pmc_fetch_$tag.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$tag -o run -- python3 $B > gpurun_out/pmc_write_$tag.log 2>&1 || exit $?
python3 scripts/prof_summary.py "$tag" lub_multi_kernel 6442457088  # (re-run locally after gpurun merges gpurun_out/)
