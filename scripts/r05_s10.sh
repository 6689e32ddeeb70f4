#!/bin/bash
# Round-5 session 10: rocprofv3 kernel traces and SQ counters of the current Orswot / Map apply
# kernels (65,536 states x 64 ops, the round-5 LDS bloom / witness-counter builds), so README and
# DESIGN quote the current code rather than round 4's traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
bash scripts/gpu.sh trace r05_oapply python3 scripts/bench_orswot_apply.py --cpu-s 0 || exit $?
bash scripts/gpu.sh trace r05_mapply python3 scripts/bench_map_apply.py || exit $?
SQ=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM,SQ_INSTS_LDS
bash scripts/gpu.sh pmc r05_oapply_sq $SQ python3 scripts/bench_orswot_apply.py --cpu-s 0 --reps 2 || exit $?
bash scripts/gpu.sh pmc r05_mapply_sq $SQ python3 scripts/bench_map_apply.py --reps 2 || exit $?
echo "session 10 done"
