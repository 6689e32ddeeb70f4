#!/bin/bash
# Map wire throughput (and the other wire workloads for the record).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/bench_wire.py --skip gcounter,pncounter,orswot > gpurun_out/bench_wire_map.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_wire_map.log
