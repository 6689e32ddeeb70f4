# Round-4 GPU session 5b: Map pair key pass with non-temporal key rows (mpnt), A/B over occupancy
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu.sh testsall tests/test_gpu_merge_batch.py -k "map"
rc=$?; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu.sh run r04_map_pair_nt_ab bash scripts/ab_tune.sh scripts/bench_merge_batch.py "--only map --steps 10" \
  mpnt=0 mpnt=1 mpnt=1,mpbpc=16 mpnt=1,mpbpc=32 mpnt=0,mpbpc=32
