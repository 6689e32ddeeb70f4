"""Summarise scripts/r05_s10.sh's apply-kernel evidence into profiles/<tag>_*.

Copies the rocprofv3 kernel stats of the Orswot / Map apply benches and reduces the SQ counter
passes to per-dispatch sums of the last profiled dispatch of each apply kernel, with
wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES and active_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES.
Usage (locally, after gpurun merged gpurun_out/): python scripts/apply_sq_summary.py r05
"""
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r05"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")
KERNELS = {"oapply": "orswot_apply_grp_kernel", "mapply": "map_apply_grp_kernel"}

out = {}
for short, kname in KERNELS.items():
    stats = os.path.join(G, f"prof_{tag}_{short}", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(P, f"{tag}_{short}_kernel_stats.csv"))
    avg = next(float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(stats)) if kname in r["Name"])
    rows = [r for r in csv.DictReader(open(os.path.join(G, f"pmc_{tag}_{short}_sq", "run_counter_collection.csv")))
            if kname in r["Kernel_Name"]]
    last = max(int(r["Dispatch_Id"]) for r in rows)
    sq = {}
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            sq[r["Counter_Name"]] = sq.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    kernel = next(r["Kernel_Name"] for r in rows)
    out[short] = {"kernel": kernel, "rocprofv3_avg_us": avg, "sq": dict(sorted(sq.items())),
                  "wait_any_frac": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
                  "active_frac": sq["SQ_ACTIVE_INST_ANY"] / sq["SQ_WAVE_CYCLES"]}
out["note"] = ("65,536 states x 64 ops (bench_orswot_apply.py / bench_map_apply.py), current build; "
               "SQ_* are per-dispatch sums of the last profiled dispatch (scripts/r05_s10.sh)")
json.dump(out, open(os.path.join(P, f"{tag}_apply_sq_counters.json"), "w"), indent=1)
print(json.dumps({k: (v["rocprofv3_avg_us"], v["wait_any_frac"], v["active_frac"]) for k, v in out.items()
                  if k != "note"}))
