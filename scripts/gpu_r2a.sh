#!/bin/bash
# Round-2 first GPU session: the whole -m gpu suite on the default library, then the Map /
# Orswot apply tests once on a CRDT_APPLY_WPE=7 build (rust-crdt_amd/build_wpe7, built on the CPU host).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
CRDT_GPU_LIB=$PWD/rust-crdt_amd/build_wpe7/libcrdt_gpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_map_apply.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_wpe7.log 2>&1
rc=$?; echo "wpe7 rc=$rc"; tail -n 25 gpurun_out/pytest_wpe7.log
exit $rc
