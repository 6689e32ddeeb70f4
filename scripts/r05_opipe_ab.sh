#!/bin/bash
# Orswot join software pipeline (CRDT_TUNE opipe=PD): the Orswot parity tests with the pipelined
# join forced on, then config 3 (65,536 x 4,096 x 64) timed with opipe = 0 / 1 / 2 / 3 in one
# process (one placement of the 128 GiB input), in two processes; parity on the last variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for pd in 1 2 3; do
  CRDT_TUNE=opipe=$pd timeout -k 10 300 python -u -m pytest tests/test_gpu_orswot.py tests/test_gpu_orswot_any_state.py \
    tests/test_gpu_kat.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_opipe_tests_$pd.log 2>&1 || exit $?
  echo "opipe=$pd tests: $(tail -n 1 gpurun_out/r05_opipe_tests_$pd.log)"
done
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/bench_orswot.py --steps 5 --tune "" opipe=1 opipe=2 opipe=3 "" opipe=2 \
    > gpurun_out/r05_opipe_ab_$rep.log 2>&1 || exit $?
  echo "== process $rep"; grep -o '"tune": "[^"]*"\|"join_ms": [0-9.]*\|"parity": "[a-z]*"' gpurun_out/r05_opipe_ab_$rep.log | paste - -
done
