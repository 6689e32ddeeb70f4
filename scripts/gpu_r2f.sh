#!/bin/bash
# Kernel breakdown of the merge_batch bench (rocprofv3 kernel trace + stats).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "${GRAFT_REPO_ROOT}/gpurun_out/prof_mb" -o mb -- python3 "${GRAFT_REPO_ROOT}/scripts/bench_merge_batch.py" --steps 3 --sample 1 > "${GRAFT_REPO_ROOT}/gpurun_out/prof_mb.log" 2>&1 || exit $?
cd "${GRAFT_REPO_ROOT}" && grep '^{' gpurun_out/prof_mb.log | cut -c1-200
find gpurun_out/prof_mb -name "*kernel_stats.csv" | head -3
