#!/bin/bash
# Map fold per-phase cycle counts (MAP_STATS build, s_memtime brackets) for the threshold scan and the round-1 scan.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for m in 1 0; do
  CRDT_GPU_LIB=$PWD/rust-crdt_amd/ab/libcrdt_gpu_stats.so CRDT_TUNE=mscan3=$m timeout -k 10 300 python -u scripts/bench_map.py --no-parity --steps 1 > gpurun_out/stats_map_scan3_$m.log 2>&1 || exit $?
  grep -h "k=" gpurun_out/stats_map_scan3_$m.log | tail -n 11
done
