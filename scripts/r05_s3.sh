#!/bin/bash
# Map fold build-variant A/B, then rocprofv3 of the counter-Map and Map<K, Orswot> benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
bash scripts/r05_map_ab.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r05_mc -o run -- python3 scripts/bench_map_counter.py --steps 5 > gpurun_out/prof_r05_mc.log 2>&1 || exit $?
grep -E "map_counter_fold" gpurun_out/prof_r05_mc/run_kernel_stats.csv | cut -c1-200
