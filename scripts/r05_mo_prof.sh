#!/bin/bash
# rocprofv3 kernel trace of the Map<K, Orswot> fold (register ring, the default) on both bench inputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for i in random causal; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mo_$i -o run -- python3 scripts/bench_map_orswot.py --input $i > gpurun_out/prof_mo_$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/prof_mo_$i.log | cut -c1-220
done
find gpurun_out/prof_mo_random gpurun_out/prof_mo_causal -name "*kernel_stats.csv" | head
