# Lattice merge_batch: flat 16-byte stream (mflat = workgroups per CU) vs the row-group kernel (mflat=0)
set -o pipefail
for t in ${TUNES:-"mflat=0" "mflat=1" "mflat=2" "mflat=0" "mflat=1"}; do
  echo "== calib $t"
  CRDT_TUNE="$t" timeout -k 10 150 python3 scripts/bench_merge_batch.py --only calib --steps 5 || exit $?
done
