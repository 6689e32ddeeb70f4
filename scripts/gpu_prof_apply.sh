cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_oapply -o run -- python3 scripts/bench_orswot_apply.py > gpurun_out/prof_oapply.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mapply -o run -- python3 scripts/bench_map_apply.py > gpurun_out/prof_mapply.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_forget -o run -- python3 scripts/bench_forget.py > gpurun_out/prof_forget.log 2>&1 || exit $?
grep -h '^{' gpurun_out/prof_oapply.log gpurun_out/prof_mapply.log gpurun_out/prof_forget.log | cut -c1-200
