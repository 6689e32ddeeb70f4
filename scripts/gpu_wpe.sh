# Variant-library A/B runner: expects rust-crdt_amd/build_<tag>/libcrdt_gpu.so built by hand (one
# object recompiled with a different constant, linked with the other objects of build/); base = the tree's library.
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in base u8 u2 base u8; do
  if [ $v = base ]; then unset CRDT_GPU_LIB; else export CRDT_GPU_LIB=$PWD/rust-crdt_amd/build_$v/libcrdt_gpu.so; fi
  echo "== $v"
  timeout -k 10 120 python -u scripts/bench_forget.py > gpurun_out/fu.log 2>&1 || exit $?
  grep '^{' gpurun_out/fu.log | grep -o '"op": "[a-z_]*"\|"kernel_us": [0-9.]*\|"parity": "[a-z]*"' | paste - - -
done
