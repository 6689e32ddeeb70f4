#!/bin/bash
# Round-6 session 21: the egress kernel pinned to 4 waves per SIMD (the K2w change took it past 128
# VGPRs): wire tests, then the value-Map ops bench twice (egress / ingest figures).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire_vmap.py tests/test_gpu_wire.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_s21_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/r06_s21_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s21_vmap_ops_$i.log 2>&1 || exit $?
  grep -h egress gpurun_out/r06_s21_vmap_ops_$i.log
done
