#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/tune_lub.py "$@" > gpurun_out/tune.log 2>&1; rc=$?
cat gpurun_out/tune.log | grep -v amdgpu.ids; exit $rc
