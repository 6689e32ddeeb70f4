bash scripts/gpu.sh run r03_oapply_fence env CRDT_TUNE=afence=1 python -u scripts/bench_orswot_apply.py && \
bash scripts/gpu.sh run r03_oapply_b python -u scripts/bench_orswot_apply.py && \
bash scripts/gpu.sh run r03_mapply_fence env CRDT_TUNE=afence=1 python -u scripts/bench_map_apply.py && \
bash scripts/gpu.sh run r03_mapply_b python -u scripts/bench_map_apply.py && \
bash scripts/gpu.sh run r03_host_orswot python -u scripts/bench_host_orswot.py
