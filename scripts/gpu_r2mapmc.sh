#!/bin/bash
# Map / Orswot apply: instruction mix per launch (SQ counters), to tell issue- from latency-bound
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc_mapply -o run -- python3 scripts/bench_map_apply.py --reps 1 > gpurun_out/pmc_mapply.log 2>&1 || { tail -5 gpurun_out/pmc_mapply.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc_oapply -o run -- python3 scripts/bench_orswot_apply.py --reps 1 > gpurun_out/pmc_oapply.log 2>&1 || { tail -5 gpurun_out/pmc_oapply.log; exit 1; }
find gpurun_out/pmc_mapply gpurun_out/pmc_oapply -name "*counter_collection.csv" | head
