#!/bin/bash
# Round-6 session 27: config 4's replicas in one contiguous device block (synth.map_replicas contig,
# bench.py --contig-input) against the torch allocator, interleaved on one box; bench_map.py beside.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for v in contig torch; do
    f=--contig-input; [ $v = torch ] && f=--no-contig-input
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-c3 --no-c5 --no-cpu-baseline $f > gpurun_out/r06_s27_bench_${v}_$rep.log 2>&1 || exit $?
    echo "bench_c4 $v $rep $(python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r06_s27_bench_${v}_$rep.log') if l.startswith('{')][0]; c=d['c4']; print(round(c['ms_per_step'],4), round(c['roofline']['avg_launch_us'],1), round(c['roofline']['frac'],4))")"
  done
done
timeout -k 10 200 python -u scripts/bench_map.py --steps 10 --cpu-replicas 16 > gpurun_out/r06_s27_map.log 2>&1 || exit $?
echo "bench_map $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/r06_s27_map.log)"
