"""Summarise a rocprofv3 kernel-trace run plus separate FETCH_SIZE / WRITE_SIZE passes for ONE
kernel (name substring) into profiles/<tag>_pmc_summary.json, and copy the kernel stats CSV.

    python scripts/prof_summary.py <tag> <kernel-substring> [algorithmic-bytes-per-launch]

Expects gpurun_out/prof_<tag>/ (--kernel-trace --stats), gpurun_out/pmc_fetch_<tag>/ and
gpurun_out/pmc_write_<tag>/ (--pmc FETCH_SIZE / --pmc WRITE_SIZE, one counter set per pass).
FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads, so it is doubled (MI355X_MICROARCH.md, HBM / rocprofv3 section)."""
import csv
import glob
import json
import os
import shutil
import sys

tag, kernel = sys.argv[1], sys.argv[2]
alg = float(sys.argv[3]) if len(sys.argv) > 3 else None
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def find(pattern):
    hits = sorted(glob.glob(os.path.join(G, pattern), recursive=True))
    return hits[0] if hits else None


out = {"kernel": kernel}
stats = find(f"prof_{tag}/**/*kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(P, f"{tag}_kernel_stats.csv"))
trace = find(f"prof_{tag}/**/*kernel_trace.csv")
if trace:
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            for r in csv.DictReader(open(trace)) if kernel in r["Kernel_Name"]]
    if durs:
        out.update(launches_traced=len(durs), avg_launch_us_rocprof=sum(durs) / len(durs),
                   min_launch_us=min(durs), max_launch_us=max(durs))


def pmc(pattern, counter):
    f = find(pattern)
    if not f:
        return []
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if kernel in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter]


fetch = pmc(f"pmc_fetch_{tag}/**/*counter_collection.csv", "FETCH_SIZE")
write = pmc(f"pmc_write_{tag}/**/*counter_collection.csv", "WRITE_SIZE")
if fetch and write:
    f_b = 2 * 1024 * sum(fetch) / len(fetch)
    w_b = 1024 * sum(write) / len(write)
    out.update(fetch_size_kib_avg=sum(fetch) / len(fetch), write_size_kib_avg=sum(write) / len(write),
               fetch_bytes_per_launch_corrected=f_b, write_bytes_per_launch=w_b, hbm_bytes_per_launch=f_b + w_b)
    if alg:
        out.update(algorithmic_bytes_per_launch=alg, traffic_over_algorithmic=(f_b + w_b) / alg)
if alg and "avg_launch_us_rocprof" in out:
    out["achieved_GBs_rocprof"] = alg / out["avg_launch_us_rocprof"] / 1e3
    out["frac_of_8TBs"] = out["achieved_GBs_rocprof"] / 8000.0
json.dump(out, open(os.path.join(P, f"{tag}_pmc_summary.json"), "w"), indent=1)
# the bench line's roofline.traffic: this checkpoint's measurement, tied to the kernel source it was
# measured on (bench.py reports null when csrc/lattice.hip no longer matches)
if kernel == "lub_multi_kernel" and "hbm_bytes_per_launch" in out:
    sys.path.insert(0, ROOT)
    import bench
    json.dump({"workload": "gcounter+pncounter lub 1048576x256", "fused": True,
               "hbm_bytes_per_launch": out["hbm_bytes_per_launch"], "source": f"profiles/{tag}_pmc_summary.json",
               "kernel_source_sha256": bench.kernel_source_sha()},
              open(os.path.join(P, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
