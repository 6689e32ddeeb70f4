# A/B of CRDT_TUNE settings on one script: bash scripts/ab_tune.sh <script.py> "<args>" <tune1> <tune2> ...
# Each setting runs twice, interleaved (placement spread shows as the spread of each pair).
set -o pipefail
script=$1; args=$2; shift 2
for rep in 1 2; do
  for t in "$@"; do
    echo "== $t (run $rep)"
    CRDT_TUNE="$t" timeout -k 10 240 python3 $script $args || exit $?
  done
done
