# Round-4 GPU session 3: the flat lattice merge stream at 1 / 2 / 4 pieces per lane, and the stream
# micro's in-place merge at 4 and 16 GiB per array (is 75% a small-array figure?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu.sh testsall tests/test_gpu_lattice.py -k merge_batch
rc=$?; [ $rc -eq 0 ] || exit $rc
TUNES="mfu=1 mfu=2 mfu=4 mflat=2,mfu=4 mflat=2,mfu=1 mfu=1 mfu=2 mfu=4" bash scripts/gpu.sh run r04_merge_flat_u bash scripts/sweep_merge_flat.sh || exit $?
bash scripts/gpu.sh run r04_stream_rate_4g timeout -k 10 200 scripts/micro/stream_rate 2 4 || exit $?
bash scripts/gpu.sh run r04_stream_rate_16g timeout -k 10 300 scripts/micro/stream_rate 2 16
