"""Summarise a rocprofv3 kernel-trace run of bench.py plus separate FETCH_SIZE / WRITE_SIZE passes
into profiles/<tag>_pmc_summary.json (one entry per bench block), copy the kernel stats CSV, and
write profiles/pmc_traffic.json (the HBM bytes per launch bench.py reports as roofline.traffic,
each entry tied to the sha256 of its kernel's source).

    python scripts/prof_summary.py <tag>

Expects gpurun_out/prof_<tag>/ (--kernel-trace --stats; its bench JSON line in
gpurun_out/prof_<tag>.log gives each block's workload and algorithmic bytes per launch),
gpurun_out/pmc_fetch_<tag>/ and gpurun_out/pmc_write_<tag>/ (--pmc FETCH_SIZE / --pmc WRITE_SIZE,
one counter set per pass).  FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE
reports half the bytes of wide coalesced streaming reads, so it is doubled (MI355X_MICROARCH.md,
HBM / rocprofv3 section)."""
import csv
import glob
import json
import os
import shutil
import sys

tag = sys.argv[1]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")
sys.path.insert(0, ROOT)
import bench  # noqa: E402

# block -> kernel-name substring of its dominant kernel
KERNELS = {"c2": "lub_multi_kernel", "c5": "lub_stream_kernel", "c3": "orswot_join_kernel", "c4": "map_fold_kernel"}


def find(pattern):
    hits = sorted(glob.glob(os.path.join(G, pattern), recursive=True))
    return hits[0] if hits else None


def bench_line():
    with open(os.path.join(G, f"prof_{tag}.log")) as f:
        lines = [ln for ln in f if ln.startswith("{")]
    return json.loads(lines[-1])


line = bench_line()
blocks = {"c2": line}
for b in ("c5", "c3", "c4"):
    if isinstance(line.get(b), dict):
        blocks[b] = line[b]

stats = find(f"prof_{tag}/**/*kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(P, f"{tag}_kernel_stats.csv"))
trace = find(f"prof_{tag}/**/*kernel_trace.csv")
trace_rows = list(csv.DictReader(open(trace))) if trace else []


def pmc(pattern, counter, kernel):
    f = find(pattern)
    if not f:
        return []
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if kernel in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter]


summary = {}
for b, blk in blocks.items():
    kernel = KERNELS[b]
    alg = float(blk["roofline"]["algorithmic_bytes_per_launch"])
    out = {"kernel": kernel, "workload": blk["config"]["workload"], "algorithmic_bytes_per_launch": alg,
           "kernel_source_sha256": bench.kernel_source_sha(b),
           "hip_event_avg_launch_us": blk["roofline"].get("avg_launch_us")}
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            for r in trace_rows if kernel in r["Kernel_Name"]]
    if durs:
        out.update(launches_traced=len(durs), avg_launch_us_rocprof=sum(durs) / len(durs),
                   min_launch_us=min(durs), max_launch_us=max(durs),
                   achieved_GBs_rocprof=alg / (sum(durs) / len(durs)) / 1e3)
        out["frac_of_8TBs"] = out["achieved_GBs_rocprof"] / 8000.0
    fetch = pmc(f"pmc_fetch_{tag}/**/*counter_collection.csv", "FETCH_SIZE", kernel)
    write = pmc(f"pmc_write_{tag}/**/*counter_collection.csv", "WRITE_SIZE", kernel)
    if fetch and write:
        f_b = 2 * 1024 * sum(fetch) / len(fetch)
        w_b = 1024 * sum(write) / len(write)
        out.update(pmc_launches=len(fetch), fetch_size_kib_avg=sum(fetch) / len(fetch),
                   write_size_kib_avg=sum(write) / len(write), fetch_bytes_per_launch_corrected=f_b,
                   write_bytes_per_launch=w_b, hbm_bytes_per_launch=f_b + w_b,
                   traffic_over_algorithmic=(f_b + w_b) / alg)
    summary[b] = out

json.dump(summary, open(os.path.join(P, f"{tag}_pmc_summary.json"), "w"), indent=1)
# the bench line's roofline.traffic: this checkpoint's measurement per block, tied to the kernel
# source it was measured on (bench.py reports null when the source no longer matches)
# (merged into the existing file: a run of some blocks keeps the other blocks' entries)
try:
    traffic = json.load(open(os.path.join(P, "pmc_traffic.json")))
except (OSError, ValueError):
    traffic = {}
for b, s in summary.items():
    if "hbm_bytes_per_launch" in s:
        traffic[b] = {"workload": s["workload"], "kernel": s["kernel"], "hbm_bytes_per_launch": s["hbm_bytes_per_launch"],
                      "source": f"profiles/{tag}_pmc_summary.json", "kernel_source_sha256": s["kernel_source_sha256"]}
if any("hbm_bytes_per_launch" in s for s in summary.values()):
    json.dump(traffic, open(os.path.join(P, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
