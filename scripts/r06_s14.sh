#!/bin/bash
# Round-6 session 14: Map<K, Orswot> fold with the 4-step ring at >= 2,048 key waves: its GPU tests,
# then bench_map_orswot.py (causal input) with the level-1 probe of a 2-range cut (the timing the
# 4-step ring reaches at 2 waves per SIMD).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map_orswot.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s14_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r06_s14_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_map_orswot.py --input causal --split-probe 2 > gpurun_out/r06_s14_mo_causal.log 2>&1 || exit $?
grep '^{' gpurun_out/r06_s14_mo_causal.log | cut -c1-400
echo "session 14 done"
