#!/bin/bash
# Counter-valued Map fold A/B: keys per wave (mckpw), the LDS-DMA ring (mcdma=8 / 16) and the
# one-key register ring (mckpw=1, the default), with the config-4 removes (P_DEF, default 0.1).
for t in ${TUNES:-"mckpw=1" "mcdma=8" "mckpw=1"}; do
  echo "== CRDT_TUNE=$t p_def=${P_DEF:-0.1}"
  CRDT_TUNE="$t" timeout -k 10 240 python3 scripts/bench_map_counter.py --parity-replicas 256 --p-def ${P_DEF:-0.1} || exit $?
done
