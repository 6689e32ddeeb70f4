#!/bin/bash
# Round-6 session 26: is config 4 slower on the final tree than at checkpoint r06e? Interleaved on one
# box: bench_map.py and bench.py's c4 block with the current library and the r06e-tree library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for v in cur r06e; do
    lib=$PWD/rust-crdt_amd/libcrdt_gpu.so; [ $v = r06e ] && lib=$PWD/rust-crdt_amd/libcrdt_gpu_r06e.so
    CRDT_GPU_LIB=$lib timeout -k 10 200 python -u scripts/bench_map.py --steps 10 --cpu-replicas 16 > gpurun_out/r06_s26_map_${v}_$rep.log 2>&1 || exit $?
    echo "bench_map $v $rep $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/r06_s26_map_${v}_$rep.log)"
    CRDT_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-c3 --no-c5 --no-cpu-baseline --causal-steps 5 > gpurun_out/r06_s26_bench_${v}_$rep.log 2>&1 || exit $?
    echo "bench_c4 $v $rep $(python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/r06_s26_bench_${v}_$rep.log') if l.startswith('{')][0]; print(round(d['c4']['ms_per_step'],4), round(d['c4']['roofline']['frac'],4))")"
  done
done
