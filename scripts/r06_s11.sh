#!/bin/bash
# Round-6 session 11: value-Map apply pass 2 with one wave per workgroup and up to 64 KiB of LDS slots:
# apply GPU tests, bench_vmap_ops at Dcap 64 twice, then a rocprofv3 kernel trace of one Dcap-64 run
# (pass 1 and pass 2 timed apart).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_map_counter_apply.py tests/test_gpu_map_orswot_apply.py tests/test_gpu_map_nested_apply.py tests/test_gpu_vmap_merge.py tests/test_gpu_wire_vmap.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06_s11_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r06_s11_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 400 python -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/r06_s11_vmap64_$rep.log 2>&1 || exit $?
  grep '^{' gpurun_out/r06_s11_vmap64_$rep.log | grep apply_batch | cut -c1-230
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r06_vmap64 -o run -- python3 -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/prof_r06_vmap64.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_r06_vmap64/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "apply" in r["Name"]:
        print(r["Name"][:90], r["Calls"], r["AverageNs"], r["MaxNs"])
PY
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r06_s11_bench.log 2>&1 || exit $?
grep -o "\"parity_detail\": {[^}]*}[^}]*}" gpurun_out/r06_s11_bench.log | head -3
echo "session 11 done"
