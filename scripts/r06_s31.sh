#!/bin/bash
# Round-6 session 31: the Orswot / Map apply benches (65,536 states x 64 ops) with their states in one
# contiguous device block against the torch allocator, interleaved on one box, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for v in contig torch; do
    f=--contig; [ $v = torch ] && f=
    timeout -k 10 300 python -u scripts/bench_orswot_apply.py --cpu-s 0 $f > gpurun_out/r06_s31_oapply_${v}_$rep.log 2>&1 || exit $?
    echo "orswot_apply $v $rep $(grep -o '"kernel_us": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/r06_s31_oapply_${v}_$rep.log | head -2 | tr '\n' ' ') $(grep -o '"parity": "[a-z]*"' gpurun_out/r06_s31_oapply_${v}_$rep.log | head -1)"
    timeout -k 10 300 python -u scripts/bench_map_apply.py $f > gpurun_out/r06_s31_mapply_${v}_$rep.log 2>&1 || exit $?
    echo "map_apply $v $rep $(grep -o '"kernel_us": [0-9.]*\|"kernel_ms": [0-9.]*' gpurun_out/r06_s31_mapply_${v}_$rep.log | head -2 | tr '\n' ' ') $(grep -o '"parity": "[a-z]*"' gpurun_out/r06_s31_mapply_${v}_$rep.log | head -1)"
  done
done
