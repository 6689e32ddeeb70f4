# Round-4 GPU session 4: sharded device-offset entry points (world 1 + world 2), the LD path with
# its scan operands in LDS (map tests in every staging mode incl. mld=1, then the A/B)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu.sh testsall tests/test_gpu_shard_abi.py tests/test_gpu_dist_world2.py tests/test_gpu_devoff.py
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu.sh testsall tests/test_gpu_map.py -k "mld or fullsize"
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu.sh run r04_map_ld2_ab bash scripts/ab_tune.sh scripts/bench_map.py "--steps 5" mld=0 mld=1
