#!/bin/bash
# Round-6: bench.py's world-2 path on this one GPU, then the rocprofv3 evidence (profiles/collect.sh).
set -o pipefail
tag=${1:-r06c}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --exchange cabi-ops --steps 5 --warmup 1 \
  --no-cpu-baseline > gpurun_out/bench_world2_$tag.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_world2_$tag.log | cut -c1-300
bash profiles/collect.sh $tag
