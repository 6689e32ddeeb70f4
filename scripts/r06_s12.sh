#!/bin/bash
# Round-6 session 12: rocprofv3 kernel trace of bench_vmap_ops at Dcap 64 (pass 1 / pass 2 apart).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r06_vmap64 -o run -- python3 -u scripts/bench_vmap_ops.py --dcap 64 > gpurun_out/prof_r06_vmap64.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_r06_vmap64/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "apply" in r["Name"]:
        print(r["Name"][:90], r["Calls"], r["AverageNs"], r["MaxNs"])
PY
echo "session 12 done"
