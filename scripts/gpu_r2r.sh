#!/bin/bash
# Map wire ingest / egress parity.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_wire_map.log 2>&1
rc=$?; tail -n 12 gpurun_out/pytest_wire_map.log; exit $rc
