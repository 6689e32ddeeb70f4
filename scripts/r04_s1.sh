# Round-4 GPU session 1: correctness of this round's changes, then the A/B measurements
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu.sh testsall tests/test_gpu_orswot_any_state.py tests/test_gpu_wide.py tests/test_gpu_mvreg.py \
  tests/test_gpu_orswot.py tests/test_gpu_lattice.py tests/test_gpu_shard_abi.py tests/test_gpu_devoff.py \
  tests/test_gpu_host_mem.py tests/test_gpu_dist_world2.py tests/test_gpu_merge_batch.py tests/test_gpu_map_apply.py \
  tests/test_gpu_orswot_apply.py tests/test_gpu_wire.py
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu.sh run r04_map_apply_pf_ab bash scripts/ab_tune.sh scripts/bench_map_apply.py "" mapf=0 mapf=1 || exit $?
bash scripts/gpu.sh run r04_orswot_apply_pf_ab bash scripts/ab_tune.sh scripts/bench_orswot_apply.py "" oapf=0 oapf=1 || exit $?
bash scripts/gpu.sh run r04_map_pair_pf_ab bash scripts/ab_tune.sh scripts/bench_merge_batch.py "--only map --steps 10" mppf=0 mppf=1 || exit $?
bash scripts/gpu.sh tests tests/test_gpu_map.py -k "mld or fullsize" || exit $?
bash scripts/gpu.sh run r04_wire_fill_ab bash scripts/ab_tune.sh scripts/bench_wire.py "--skip gcounter,pncounter,map" wfill=0 wfill=1 || exit $?
bash scripts/gpu.sh run r04_map_ld_ab bash scripts/ab_tune.sh scripts/bench_map.py "--steps 5" mld=0 mld=1 || exit $?
bash scripts/gpu.sh run r04_merge_flat bash scripts/sweep_merge_flat.sh
