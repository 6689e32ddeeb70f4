#!/usr/bin/env python3
"""Benchmark: batched CvRDT lub (replica-merges/s) on MI355X — BASELINE.json config 2.

One step = the two lubs of config 2 over HBM-resident synthetic replicas:
    GCounter  lub_many of 1,048,576 replicas x 256 actors (u64)       2 GiB read
    PNCounter lub_many of 1,048,576 replicas x (2 x 256) actors (u64)  4 GiB read
= 2,097,152 replica-merges per rank per step.  With --gpus N (torchrun, one process per GPU)
every rank holds its own 1M-replica shard of one global input (weak scaling) and the step ends
with the one real exchange of the path: an unsigned-max all-reduce of the 768-word partial
lubs over RCCL.  value = replica-merges of all ranks / max-over-ranks wall time.

The JSON line also carries
  roofline      the dominant kernel (lub_stream_kernel, both launches of the step), its
                average launch duration from HIP events on the launch stream vs the algorithmic
                bytes per launch, against 8 TB/s;
  cpu_baseline  the oracle's restated reference fold (VClock::merge over ordered maps) on a
                bounded sample of the same workload, split over the host's threads (up to 16),
                plus the one-thread figure (rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rust-crdt_amd"))

R_REPLICAS = 1 << 20
A_ACTORS = 256
SEED_G, SEED_P = 0x5EED0002, 0x5EED0003
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--replicas", type=int, default=R_REPLICAS, help="replicas per rank (config 2: 1M)")
    ap.add_argument("--actors", type=int, default=A_ACTORS)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="target fold seconds of the CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm) for real runs; gloo lets several ranks share one GPU in tests")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC-derived HBM bytes per launch (written by profiles/collect.sh)")
    return ap.parse_args()


def cpu_threads():
    """Host threads for the CPU baseline: the CPUs this process may run on, at most 16 (the
    GPU box's CPU share; os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(args):
    """Restated reference fold (oracle, 'port'): VClock::merge (vclock.rs:130-136) over ordered
    maps for GCounter rows and P/N pairs for PNCounter rows, on a bounded sample of the same
    synthetic input — split over the host's threads (partials merged at the end, SURVEY §8d
    CPU timing (2)), and on one thread for reference."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    T = cpu_threads()

    def run(threads, per_thread, seconds):
        done_rows, fold_s, reps = 0, 0.0, 0
        t_start = time.time()
        while fold_s < seconds and time.time() - t_start < 4 * seconds:
            n = per_thread * threads
            row0 = reps * n
            g = O.synth_matrix(SEED_G, n, args.actors, 0, row0=row0)
            _, tg = O.counter_fold_mt(g, False, threads)
            p = O.synth_matrix(SEED_P, n, 2 * args.actors, 0, row0=row0)
            _, tp = O.counter_fold_mt(p, True, threads)
            fold_s += tg + tp
            done_rows += 2 * n
            reps += 1
        return done_rows / fold_s, reps, fold_s

    v1, reps1, s1 = run(1, 16384, args.cpu_seconds / 2)
    vT, repsT, sT = run(T, 4096, args.cpu_seconds)
    return {
        "value": vT,
        "unit": "replica-merges/s",
        "cores": T,
        "kind": "port",
        "sample": (f"{repsT} x ({T}x4096 GCounter x {args.actors} + {T}x4096 PNCounter x 2x{args.actors}) replicas "
                   f"of the same synthetic input, left fold of the restated VClock::merge over std::map "
                   f"(oracle/ref_fold.cpp) split over {T} threads + final merge of the partials, map ingest "
                   f"excluded; {sT:.2f} s of fold"),
        "single_core": {"value": v1, "cores": 1, "sample": f"{reps1} x (16384 + 16384) replicas, {s1:.2f} s of fold"},
    }


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import crdts_gpu as cg
    from crdts_gpu import dist as cdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = local % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)
    ctx = cg.Context.default(dev)

    R, A = args.replicas, args.actors
    # Synthetic replicas, generated in HBM; rank k owns rows [k*R, (k+1)*R) of the global input.
    g_in = torch.empty((R, A), dtype=torch.int64, device="cuda")
    p_in = torch.empty((R, 2 * A), dtype=torch.int64, device="cuda")
    cg.synth_fill(ctx, g_in, SEED_G, 0, first_row=rank * R)
    cg.synth_fill(ctx, p_in, SEED_P, 0, first_row=rank * R)
    g_out = torch.empty((A,), dtype=torch.int64, device="cuda")
    p_out = torch.empty((2 * A,), dtype=torch.int64, device="cuda")
    both = torch.empty((3 * A,), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step():
        cg.gcounter.lub_many(g_in, out=g_out, ctx=ctx)
        cg.pncounter.lub_many(p_in, out=p_out, ctx=ctx)
        if world > 1:
            both[:A].copy_(g_out)
            both[A:].copy_(p_out)
            cdist.allreduce_umax_(both)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ctx.timing_reset()
    ctx.set_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    kern_ms, launches = ctx.timing("lub_stream")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Parity (outside the timed region): unsigned max with torch ops + sampled CPU rows.
    sign = torch.tensor(-(2**63), dtype=torch.int64, device="cuda")
    ref_g, ref_p = (g_in ^ sign).amax(0) ^ sign, (p_in ^ sign).amax(0) ^ sign
    if world > 1:  # the exchanged result must equal the max of every rank's torch reference
        ref = torch.cat([ref_g, ref_p])
        cdist.allreduce_umax_(ref)
        ok = bool(torch.equal(both, ref))
        t_ok = torch.tensor([1 if ok else 0], dtype=torch.int64, device="cuda")
        dist.all_reduce(t_ok, op=dist.ReduceOp.MIN)
        ok = bool(t_ok.item())
    else:
        ok = bool(torch.equal(g_out, ref_g)) and bool(torch.equal(p_out, ref_p))

    merges_per_step = 2 * R * world
    value = merges_per_step * args.steps / elapsed
    bytes_per_step = (R * A * 8 + A * 8) + (R * 2 * A * 8 + 2 * A * 8)
    avg_launch_bytes = bytes_per_step / 2
    avg_launch_s = (kern_ms / 1e3) / launches if launches else float("nan")
    achieved = avg_launch_bytes / avg_launch_s / 1e9
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if tj.get("workload") == f"gcounter+pncounter lub {R}x{A}":
            traffic = tj.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    if rank == 0:
        out = {
            "metric": "replica-merges/sec (whole node) + achieved HBM GB/s as % of MI355X peak",
            "value": value,
            "unit": "replica-merges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (counter-based splitmix64 replicas generated in HBM, seeds 0x5EED0002/3)",
            "config": {
                "workload": f"gcounter+pncounter lub {R}x{A}",
                "replicas_per_gpu": R,
                "actors": A,
                "types": ["GCounter (A u64)", "PNCounter (2A u64)"],
                "replica_merges_per_step": merges_per_step,
                "exchange": "RCCL all-reduce MAX (sign-biased u64) of 3A words" if world > 1 else "none",
                "parallelism": f"replica-shard x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "lub_stream_kernel<Max,2,8> (GCounter + PNCounter launches)",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "avg_launch_us": avg_launch_s * 1e6,
                "launches": launches,
                "algorithmic_bytes_per_launch": avg_launch_bytes,
            },
            "cpu_baseline": None,
            "parity": "ok" if ok else "MISMATCH",
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
