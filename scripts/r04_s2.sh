# Round-4 GPU session 2: apply-kernel changes (Map entry-row prefetch, one-write new slots),
# A/B against the previous build, rocprofv3 kernel stats and SQ counters of both apply kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu.sh testsall tests/test_gpu_orswot_apply.py tests/test_gpu_map_apply.py tests/test_gpu_merge_batch.py
rc=$?; [ $rc -eq 0 ] || exit $rc
ab() {  # ab <tag> <script>: previous vs current library, interleaved twice
  for rep in 1 2; do
    for lib in prev cur; do
      l=rust-crdt_amd/libcrdt_gpu.so; [ $lib = prev ] && l=rust-crdt_amd/libcrdt_gpu_prev.so
      echo "== $lib (run $rep)"
      CRDT_GPU_LIB=$PWD/$l timeout -k 10 240 python3 $2 || return $?
    done
  done
}
ab oapply scripts/bench_orswot_apply.py > gpurun_out/r04_oapply_ab.log 2>&1 || exit $?
ab mapply scripts/bench_map_apply.py > gpurun_out/r04_mapply_ab.log 2>&1 || exit $?
bash scripts/ab_tune.sh scripts/bench_orswot_apply.py "" ohpf=0 ohpf=1 > gpurun_out/r04_oapply_hpf_ab.log 2>&1 || exit $?
grep -h -o '^== .*\|"kernel_us": [0-9.]*' gpurun_out/r04_oapply_ab.log gpurun_out/r04_mapply_ab.log gpurun_out/r04_oapply_hpf_ab.log
bash scripts/gpu.sh trace r04_oapply python3 scripts/bench_orswot_apply.py || exit $?
bash scripts/gpu.sh trace r04_mapply python3 scripts/bench_map_apply.py || exit $?
SQ=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM,SQ_INSTS_LDS,SQ_WAIT_INST_ANY
bash scripts/gpu.sh pmc r04_oapply_sq $SQ python3 scripts/bench_orswot_apply.py || exit $?
bash scripts/gpu.sh pmc r04_mapply_sq $SQ python3 scripts/bench_map_apply.py
