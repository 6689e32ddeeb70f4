#!/bin/bash
# Round-6 session 1: (a) the HBM ceiling of config 4's access pattern (scripts/micro/map_stream.hip:
# one vs two waves per key, a stand-in test cost per chunk); (b) config 3's roofline evidence from
# ONE bench.py c3 run per pass: rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE passes, each of a
# bench.py run with the contiguous-block input, so the profile and the bench line share a box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
(hostname; rocm-smi --showuniqueid --showserial 2>&1) > gpurun_out/r06_s1_box.txt || true
bash scripts/gpu.sh run r06_map_stream ./scripts/micro/map_stream || exit $?
B="bench.py --steps 3 --warmup 1 --causal-steps 5 --no-c5 --no-c4 --no-cpu-baseline"
bash scripts/gpu.sh trace r06_c3 python3 $B || exit $?
bash scripts/gpu.sh pmc r06_c3_fetch FETCH_SIZE python3 $B || exit $?
bash scripts/gpu.sh pmc r06_c3_write WRITE_SIZE python3 $B || exit $?
echo "session 1 done"
