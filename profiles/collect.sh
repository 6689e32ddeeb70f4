#!/bin/bash
# Collect the rocprofv3 evidence for bench.py's blocks (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command     -> gpurun_out/prof_<tag>/ (+ its JSON line)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2)
# The command runs every block (c2 head, c5, c3, c4), so one set of passes covers the dominant
# kernel of each: lub_multi_kernel, lub_stream_kernel, orswot_join_kernel, map_fold_kernel.
# Then (locally, after gpurun merges gpurun_out/) scripts/prof_summary.py <tag> writes
# profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc_summary.json and profiles/pmc_traffic.json.
tag=${1:-r05}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --no-cpu-baseline"  # (the bench line's own step / warm-up counts, so the averages match its blocks)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 $B > gpurun_out/prof_$tag.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- python3 $B > gpurun_out/pmc_fetch_$tag.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$tag -o run -- python3 $B > gpurun_out/pmc_write_$tag.log 2>&1 || exit $?
echo "collected $tag"
