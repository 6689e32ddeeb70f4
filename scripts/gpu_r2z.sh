#!/bin/bash
# Map fold (config 4) rocprofv3 evidence for the RS path (default) and the LDS-DMA ring (mrs=0):
# kernel trace + stats, FETCH_SIZE pass, WRITE_SIZE pass (separate passes).
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for v in rs dma; do
  if [ $v = dma ]; then export CRDT_TUNE=mrs=0; else unset CRDT_TUNE; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mapprof_$v -o run -- python3 scripts/prof_map.py > gpurun_out/mapprof_$v.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/mappmc_fetch_$v -o run -- python3 scripts/prof_map.py > gpurun_out/mappmc_fetch_$v.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/mappmc_write_$v -o run -- python3 scripts/prof_map.py > gpurun_out/mappmc_write_$v.log 2>&1 || exit $?
  echo "$v done"
done
