#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Stops at the first step that faults / aborts / times out (exit >= 2 and != pytest's 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests smoke bench prof}"
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python -u bench.py --steps 20 --warmup 3 ;;
    prof)  run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    apply) run bench_apply 300 python -u scripts/bench_orswot_apply.py ;;
    mapapply) run bench_mapapply 300 python -u scripts/bench_map_apply.py ;;
    forget) run bench_forget 300 python -u scripts/bench_forget.py ;;
    causal) run bench_causal 300 python -u scripts/bench_causal.py ;;
  esac
done
echo "== all done"
