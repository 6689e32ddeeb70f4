#!/bin/bash
# Round-6 session 29: the Map<K, Orswot> fold at config-4 scale with its replicas in one contiguous
# device block against the torch allocator (random and causal inputs), interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for inp in random causal; do
  for v in contig torch; do
    f=--contig; [ $v = torch ] && f=
    timeout -k 10 300 python -u scripts/bench_map_orswot.py --input $inp --parity-replicas 64 $f > gpurun_out/r06_s29_${inp}_$v.log 2>&1 || exit $?
    echo "$inp $v $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/r06_s29_${inp}_$v.log) $(grep -o '"parity": "[a-z]*"' gpurun_out/r06_s29_${inp}_$v.log)"
  done
done
