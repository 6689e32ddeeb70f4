# A/B: Orswot apply with the slots' witness counters in LDS (default build) vs without (CRDT_OA_WITV=0)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orswot_apply.py > gpurun_out/witv_tests.log 2>&1; rc=$?; tail -2 gpurun_out/witv_tests.log; [ $rc = 0 ] || exit $rc
R=$PWD/rust-crdt_amd
for rep in 1 2 3; do
 for L in libcrdt_gpu.so build_var_nowitv/libcrdt_gpu.so; do
  for m in "0.2 0.3" "0.2 0"; do set -- $m
   echo -n "lib=$L mix=$1,$2 "; CRDT_GPU_LIB=$R/$L timeout -k 10 150 python -u scripts/bench_orswot_apply.py --p-rm $1 --p-future $2 --cpu-s 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_us'],1), d['parity'])" || exit 1
  done
 done
done
