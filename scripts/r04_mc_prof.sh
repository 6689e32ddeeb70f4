#!/bin/bash
# Counter-valued Map fold: the default run (config-4 removes), no removes, then SQ counters (one
# pass) on the default run (bench_map_counter --steps 1).
echo "== default"
timeout -k 10 240 python3 scripts/bench_map_counter.py || exit $?
echo "== p_def=0"
timeout -k 10 240 python3 scripts/bench_map_counter.py --parity-replicas 128 --p-def 0 || exit $?
SQ=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM,SQ_INSTS_LDS,SQ_WAIT_INST_ANY
bash scripts/gpu.sh pmc r04_mcounter_sq $SQ python3 scripts/bench_map_counter.py --steps 1 --parity-replicas 64
