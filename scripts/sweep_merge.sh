# Concurrency sweep of the pairwise merge / forget streams (CRDT_TUNE knobs)
set -o pipefail
for t in "pocc=0" "pocc=1" "pocc=1,prows=64" "pocc=1,prows=256" "pocc=2,pur=4" "pocc=1"; do
  echo "== orswot $t"
  CRDT_TUNE="$t" timeout -k 10 150 python3 scripts/bench_merge_batch.py --only orswot --steps 5 --sample 2 || exit $?
done
for t in "mpbpc=16" "mpbpc=8" "mpbpc=4" "mpbpc=2" "mpbpc=1"; do
  echo "== map $t"
  CRDT_TUNE="$t" timeout -k 10 150 python3 scripts/bench_merge_batch.py --only map --steps 5 --sample 2 || exit $?
done
for t in "rbpc=4" "rbpc=2" "rbpc=1" "rbpc=8"; do
  echo "== forget $t"
  CRDT_TUNE="$t" timeout -k 10 200 python3 scripts/bench_forget.py || exit $?
done
