# Map merge_batch key pass: workgroups per CU A/B (CRDT_TUNE mpbpc), each after the full bench's
# earlier allocations (calibration + Orswot pass) so the placement matches bench_merge_batch.py
set -o pipefail
for t in "mpbpc=16" "mpbpc=64" "mpbpc=16" "mpbpc=64"; do
  echo "== map $t"
  CRDT_TUNE="$t" timeout -k 10 200 python3 scripts/bench_merge_batch.py --steps 5 --sample 2 || exit $?
done
