#!/bin/bash
# bench.py N>1 code paths on one GPU (gloo): the fused torch exchange, and --exchange cabi whose
# RCCL communicator setup fails on a shared GPU ("duplicate GPU") so every rank falls back together.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --exchange torch --dist-backend gloo --steps 3 --warmup 1 --replicas 65536 --no-cpu-baseline > gpurun_out/bench_w2_fused.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_w2_fused.log | cut -c1-200
timeout -k 10 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --exchange cabi --dist-backend gloo --steps 3 --warmup 1 --replicas 65536 --no-cpu-baseline > gpurun_out/bench_w2_cabi_fallback.log 2>&1 || exit $?
grep -h 'comm_init failed\|^{' gpurun_out/bench_w2_cabi_fallback.log | cut -c1-300
