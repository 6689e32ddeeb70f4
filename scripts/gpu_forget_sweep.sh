cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for t in rbpc=8 rbpc=8 rbpc=8 rbpc=2,mfv2=0 rbpc=2,mfv2=0 rbpc=2,mfv2=0 rbpc=8,mfv2=0 rbpc=8,mfv2=0; do
  echo "== $t"
  CRDT_TUNE=$t timeout -k 10 120 python -u scripts/bench_forget.py > gpurun_out/fs.log 2>&1 || exit $?
  grep '^{' gpurun_out/fs.log | cut -c1-150
done
