# Round-4 checkpoint, part 2 (part 1 = the full `-m gpu` suite): smoke(), bench.py at N=1, the
# rocprofv3 evidence of its dominant kernel (profiles/collect.sh), then bench.py's N > 1 code path at
# world 2 on this one GPU (gloo + the C ABI's caller-collectives seam: exchange / agree times).
set -o pipefail
tag=${1:-r04a}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke_$tag.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$tag.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_$tag.log | cut -c1-600
bash profiles/collect.sh "$tag" || exit $?
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --exchange cabi-ops --steps 5 --warmup 1 \
  --no-cpu-baseline > gpurun_out/bench_world2_$tag.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_world2_$tag.log | cut -c1-1500
bash scripts/gpu.sh trace r04_oapply_def python3 scripts/bench_orswot_apply.py
