#!/bin/bash
# rocprofv3 evidence for the Map fold (config 4) and the causal-helper kernels: kernel trace +
# stats, then FETCH_SIZE and WRITE_SIZE passes over the Map bench (separate passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
M="scripts/bench_map.py --no-parity --steps 3"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_map -o run -- python3 $M > gpurun_out/prof_map.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_causal -o run -- python3 scripts/bench_causal.py > gpurun_out/prof_causal.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_map -o run -- python3 $M > gpurun_out/pmc_fetch_map.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_map -o run -- python3 $M > gpurun_out/pmc_write_map.log 2>&1 || exit $?
echo "== all done"
