"""Summarise rocprofv3 outputs of profiles/collect.sh into profiles/<tag>_* files."""
import csv
import glob
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")
KERNELS = ("lub_stream_kernel", "lub_multi_kernel")  # per-lub launches / the fused step launch


def find(pattern):
    hits = sorted(glob.glob(os.path.join(G, pattern), recursive=True))
    return hits[0] if hits else None


stats = find(f"prof_{tag}/**/*kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(P, f"{tag}_kernel_stats.csv"))
trace = find(f"prof_{tag}/**/*kernel_trace.csv")
durs = []
if trace:
    for r in csv.DictReader(open(trace)):
        if any(k in r["Kernel_Name"] for k in KERNELS):
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def pmc(pattern, counter):
    f = find(pattern)
    vals = []
    if not f:
        return vals
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if any(k in name for k in KERNELS) and r.get("Counter_Name") == counter:
            vals.append(float(r["Counter_Value"]))
    return vals


fetch = pmc(f"pmc_fetch_{tag}/**/*counter_collection.csv", "FETCH_SIZE")
write = pmc(f"pmc_write_{tag}/**/*counter_collection.csv", "WRITE_SIZE")
summary = {"kernel": "/".join(KERNELS), "launches_traced": len(durs)}
if durs:
    summary["avg_launch_us_rocprof"] = sum(durs) / len(durs)
if fetch and write:
    # FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
    # coalesced streaming reads (MI355X_MICROARCH.md:298), so it is doubled.
    f_b = 2 * 1024 * sum(fetch) / len(fetch)
    w_b = 1024 * sum(write) / len(write)
    summary.update({"fetch_size_kib_avg": sum(fetch) / len(fetch), "write_size_kib_avg": sum(write) / len(write),
                    "hbm_bytes_per_launch": f_b + w_b, "fetch_bytes_per_launch_corrected": f_b,
                    "write_bytes_per_launch": w_b})
bench = None
for line in open(os.path.join(G, f"prof_{tag}.log")) if os.path.exists(os.path.join(G, f"prof_{tag}.log")) else []:
    if line.startswith("{"):
        bench = json.loads(line)
if bench:
    summary["workload"] = bench["config"]["workload"]
    summary["fused"] = bench["config"].get("launches_per_step", 2) == 1
    summary["algorithmic_bytes_per_launch"] = bench["roofline"]["algorithmic_bytes_per_launch"]
    summary["avg_launch_us_hip_events"] = bench["roofline"]["avg_launch_us"]
json.dump(summary, open(os.path.join(P, f"{tag}_pmc_summary.json"), "w"), indent=1)
if "hbm_bytes_per_launch" in summary and bench:
    json.dump({"workload": summary["workload"], "fused": summary["fused"],
               "hbm_bytes_per_launch": summary["hbm_bytes_per_launch"],
               "source": f"profiles/{tag}_pmc_summary.json"}, open(os.path.join(P, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
