# FETCH_SIZE and WRITE_SIZE passes (separate runs) over the forget bench.
cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_forget -o run -- python3 scripts/bench_forget.py > gpurun_out/pmc_fetch_forget.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_forget -o run -- python3 scripts/bench_forget.py > gpurun_out/pmc_write_forget.log 2>&1 || exit $?
echo "== all done"
