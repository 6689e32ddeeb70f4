#!/bin/bash
# Round-6 session 28: the default bench (contiguous c4 input, parity + CPU legs), then the rocprofv3
# evidence of the same build (kernel trace + FETCH / WRITE passes, profiles/collect.sh r06j).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r06j.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_r06j.log | cut -c1-300
bash profiles/collect.sh r06j
