#!/bin/bash
# Final round-2 checkpoint: the whole round checkpoint, then rocprofv3 kernel stats of the apply benches
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
bash scripts/gpu_round.sh r02l || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mapply_r02l -o run -- python3 scripts/bench_map_apply.py > gpurun_out/prof_mapply_r02l.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_oapply_r02l -o run -- python3 scripts/bench_orswot_apply.py > gpurun_out/prof_oapply_r02l.log 2>&1 || exit $?
grep -h '^{' gpurun_out/prof_mapply_r02l.log gpurun_out/prof_oapply_r02l.log | cut -c1-200
