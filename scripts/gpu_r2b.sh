#!/bin/bash
# New round-2 GPU tests (world-2 real kernels, full-size configs 3/4, even-A Map shapes), then the
# Map apply bench on the default and the CRDT_APPLY_WPE=7 library (A/B x2).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_golden_synth.py tests/test_gpu_orswot.py tests/test_gpu_map.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_new.log | tail -n 30
[ $rc -ne 0 ] && exit $rc
for v in base wpe7 base wpe7; do
  if [ $v = base ]; then unset CRDT_GPU_LIB; else export CRDT_GPU_LIB=$PWD/rust-crdt_amd/build_$v/libcrdt_gpu.so; fi
  echo "== $v"
  timeout -k 10 180 python -u scripts/bench_map_apply.py > gpurun_out/mapply_$v.log 2>&1 || exit $?
  grep '^{' gpurun_out/mapply_$v.log | tail -n 2
done
