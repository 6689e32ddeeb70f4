cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for t in hot=4 hot=6 hot=8 hot=3; do
  echo "== $t"
  CRDT_TUNE=$t timeout -k 10 120 python -u scripts/bench_orswot_apply.py > gpurun_out/hs.log 2>&1 || exit $?
  grep '^{' gpurun_out/hs.log | grep -o '"kernel_us": [0-9.]*\|"parity": "[a-z]*"' | paste - -
done
