mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_orswot_apply.py tests/test_gpu_map_apply.py > gpurun_out/meta_tests.log 2>&1; rc=$?; tail -2 gpurun_out/meta_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do
 for t in "" oameta=0; do echo -n "orswot tune=$t "; timeout -k 10 150 python -u scripts/bench_orswot_apply.py --tune "$t" --cpu-s 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_us'],1), d['parity'])" || exit 1; done
 for t in "" mameta=0; do echo -n "map tune=$t "; timeout -k 10 200 python -u scripts/bench_map_apply.py --tune "$t" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['kernel_us'],1), d['parity'], d['deferred_left'])" || exit 1; done
done
