#!/bin/bash
# Map<K, Orswot> bench, then the counter Map's keys-per-wave option where keys outnumber SIMDs
# (4,096 keys x 4,096 replicas: 4 key waves per SIMD at one key per wave).
timeout -k 10 300 python3 scripts/bench_map_orswot.py || exit $?
for t in mckpw=1 mckpw=2 mckpw=1; do
  echo "== CRDT_TUNE=$t keys=4096"
  CRDT_TUNE="$t" timeout -k 10 240 python3 scripts/bench_map_counter.py --keys 4096 --replicas 4096 --parity-replicas 64 || exit $?
done
echo "== config-4 shape, ring depth after the unclamped ring"
TUNES="mcdep=8 mcdep=16 mcdep=8" bash scripts/ab_map_counter.sh || exit $?
