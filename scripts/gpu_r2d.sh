#!/bin/bash
# Host-memory mode tests + throughput, merge_batch throughput (config-3/4 shapes), and the Map
# forget spread experiment (separate vs one-slab buffers, 3 processes each, alternating).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_mem.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_host_mem.log 2>&1
rc=$?; tail -n 25 gpurun_out/pytest_host_mem.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_host_mem.py > gpurun_out/bench_host_mem.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_host_mem.log
timeout -k 10 400 python -u scripts/bench_merge_batch.py > gpurun_out/bench_merge_batch.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_merge_batch.log
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --tag p$i > gpurun_out/spread_sep_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u scripts/bench_forget_spread.py --slab --tag p$i > gpurun_out/spread_slab_$i.log 2>&1 || exit $?
  grep -h '^{' gpurun_out/spread_sep_$i.log gpurun_out/spread_slab_$i.log | cut -c1-220
done
