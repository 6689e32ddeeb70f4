#!/bin/bash
# Counter Map fold with the automatic keys-per-wave rule: config-4 shape (1,024 keys: one key per
# wave) and 4,096 keys x 4,096 replicas (two keys per wave).
timeout -k 10 240 python3 scripts/bench_map_counter.py || exit $?
timeout -k 10 240 python3 scripts/bench_map_counter.py --keys 4096 --replicas 4096 --parity-replicas 64
