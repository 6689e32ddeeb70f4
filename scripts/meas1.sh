bash scripts/gpu.sh run r03_glds ./scripts/micro/glds_rate && \
bash scripts/gpu.sh run r03_map python -u scripts/bench_map.py && \
bash scripts/gpu.sh run r03_oapply python -u scripts/bench_orswot_apply.py && \
bash scripts/gpu.sh run r03_mapply python -u scripts/bench_map_apply.py && \
bash scripts/gpu.sh run r03_wire python -u scripts/bench_wire.py --skip gcounter,pncounter
