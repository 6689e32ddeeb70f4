# Round-4 GPU session 5: Map pair key pass storing only changed rows (mpsk), A/B + PMC write bytes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu.sh testsall tests/test_gpu_merge_batch.py tests/test_gpu_wide.py -k "map"
rc=$?; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu.sh run r04_map_pair_skip_ab bash scripts/ab_tune.sh scripts/bench_merge_batch.py "--only map --steps 10" mpsk=0 mpsk=1 || exit $?
CRDT_TUNE=mpsk=1 bash scripts/gpu.sh pmc r04_map_pair_write WRITE_SIZE python3 scripts/bench_merge_batch.py --only map --steps 3 || exit $?
CRDT_TUNE=mpsk=1 bash scripts/gpu.sh pmc r04_map_pair_fetch FETCH_SIZE python3 scripts/bench_merge_batch.py --only map --steps 3
