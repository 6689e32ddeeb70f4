#!/bin/bash
# Map fold FETCH_SIZE with and without the non-temporal step-image loads.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out/pmc_mnt && export TMPDIR=/tmp
for m in 0 1; do
  CRDT_TUNE=mnt=$m timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex map_fold --output-format csv -d gpurun_out/pmc_mnt/m$m -o run -- python3 scripts/prof_map.py > gpurun_out/pmc_mnt/m$m.log 2>&1 || exit $?
  tail -1 gpurun_out/pmc_mnt/m$m.log
done
find gpurun_out/pmc_mnt -name "*counter_collection.csv"
