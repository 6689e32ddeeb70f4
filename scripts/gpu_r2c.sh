#!/bin/bash
# Sharded C-ABI tests at world 1, bench c2 / c5 at N=1, and the bench's N>1 code path at world 2 on
# one GPU (torch exchange over gloo: RCCL refuses two ranks per GPU).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_shard.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_shard.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_c2.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -n 1 gpurun_out/bench_c5.log
timeout -k 10 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --exchange torch --dist-backend gloo --steps 3 --warmup 1 --replicas 65536 --no-cpu-baseline > gpurun_out/bench_w2.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_w2.log
