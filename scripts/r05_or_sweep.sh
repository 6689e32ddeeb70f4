#!/bin/bash
# Config-3 Orswot join: join geometry variants inside one process (one physical placement of the
# 128 GiB input), in 3 processes (placements), to see which geometry is robust to placement.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do
  timeout -k 10 300 python -u scripts/bench_orswot.py --steps 4 --tune "" ompt=8 ompt=16 obpc=1 obpc=3 ounroll=2 "" > gpurun_out/r05_or_sweep_$rep.log 2>&1 || exit $?
  echo "== process $rep"; grep -o '"tune": "[^"]*"\|"join_ms": [0-9.]*' gpurun_out/r05_or_sweep_$rep.log | paste - - 
done
