#!/bin/bash
# Map fold with the minus-one mirror copies: parity (all staging / scan modes) and A/B against the
# previous build (rust-crdt_amd/ab/libcrdt_gpu_base.so via CRDT_GPU_LIB), alternating.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_map.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_map_dec.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_dec.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q -k map --timeout 280 --timeout-method thread > gpurun_out/pytest_map_full_dec.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_map_full_dec.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 10 > gpurun_out/bench_map_dec_$i.log 2>&1 || exit $?
  CRDT_GPU_LIB=$PWD/rust-crdt_amd/ab/libcrdt_gpu_base.so timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 10 > gpurun_out/bench_map_base_$i.log 2>&1 || exit $?
  for f in gpurun_out/bench_map_dec_$i.log gpurun_out/bench_map_base_$i.log; do
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[1], round(d['kernel_ms'],4), round(d['frac_of_8TBs'],4))" $f
  done
done
