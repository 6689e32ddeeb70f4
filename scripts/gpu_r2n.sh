#!/bin/bash
# Multi-segment lub: parity, then bench A/B fused vs per-lub launches (alternating, 3 each).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lattice_multi.py tests/test_gpu_lattice.py tests/test_gpu_shard_abi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_multi.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --fused > gpurun_out/bench_fused_$i.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-fused > gpurun_out/bench_sep_$i.log 2>&1 || exit $?
  python3 -c "
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['roofline']
    print(f, round(d['value']/1e9,4), 'e9', round(d['ms_per_step'],4), 'ms', round(r['frac'],4), round(r['avg_launch_us'],1), r['launches'])
" gpurun_out/bench_fused_$i.log gpurun_out/bench_sep_$i.log
done
