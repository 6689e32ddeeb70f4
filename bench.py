#!/usr/bin/env python3
"""Benchmark: batched CvRDT lub (replica-merges/s) on MI355X — BASELINE.json config 2 (`value`) and
config 5 (the `c5` block of the same line).

--workload c2 (default): one step = the two lubs of config 2 over HBM-resident synthetic replicas:
    GCounter  lub_many of 1,048,576 replicas x 256 actors (u64)       2 GiB read
    PNCounter lub_many of 1,048,576 replicas x (2 x 256) actors (u64)  4 GiB read
= 2,097,152 replica-merges per rank per step.  The same line then carries a `c5` block: one step =
one GPU's shard of config 5, VClock lub_many of 1,048,576 replicas x 1,024 actors (8 GiB read; at
--gpus 8 the global input is config 5's 8M replicas and the exchange its RCCL max all-reduce).
--workload c5: config 5 as the headline instead (no second block).
At N = 1 the line also carries `c3` and `c4` blocks (--no-c3 / --no-c4 drop them): BASELINE config 3,
Orswot<u64, u32> lub_many of 65,536 replicas x 4,096 members x 64 actors with deferred removes (128 GiB
of entries), and config 4, Map<u32, MVReg<u64>> lub_many of 16,384 replicas x 1,024 keys x 32 actors,
V = 2 (12.25 GiB), both generated in HBM; one step = one whole lub_many (every kernel of it), the
roofline is its dominant kernel (orswot_join_kernel / map_fold_kernel), and the oracle leg (rank 0,
N = 1) checks the result on a member / key sample and times the restated reference fold on a replica
subsample.

--gpus N > 1: one process per GPU.  Started without WORLD_SIZE, the script starts its own
`python -m torch.distributed.run --nproc-per-node N` child BEFORE touching the GPU, relays rank 0's
JSON line and exits with the child's status; under torchrun, WORLD_SIZE must equal --gpus.  Every
rank holds its own 1M-replica shard of one global input (weak scaling) and each lub of the step is
the C ABI's own sharded entry point (crdt_lub_many_multi_sharded / crdt_vclock_lub_many_sharded:
local lub + ONE ncclAllReduce(ncclUint64, ncclMax) over the ctx's RCCL communicator, the path a Rust
caller without torch.distributed takes; torch.distributed only ships the 128-byte unique id and
runs the barriers).  --exchange cabi-ops runs the same C code over crdt_ctx_comm_init_ops with
torch.distributed host callbacks (gloo: several ranks on one GPU); --exchange torch the
torch.distributed twin.  value = replica-merges of all ranks / max-over-ranks wall time.

The JSON line also carries
  step_ms       median / min / max of the per-step durations (HIP events around every step on the
                launch stream, max over ranks per step); ms_per_step is the wall-clock mean
  roofline      the dominant kernel, its average launch duration from HIP events on the launch
                stream vs the algorithmic bytes per launch, against 8 TB/s
  cpu_baseline  the oracle's restated reference fold (VClock::merge over ordered maps) on a
                bounded sample of the same workload, split over the host's threads (up to 16),
                plus the one-thread figure (rank 0 at N=1 only).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rust-crdt_amd"))

R_REPLICAS = 1 << 20
A_ACTORS = 256
A_C5 = 1024
SEED_G, SEED_P, SEED_V = 0x5EED0002, 0x5EED0003, 0x5EED0005
HBM_PEAK_GBS = 8000.0
METRIC = "replica-merges/sec (whole node) + achieved HBM GB/s as % of MI355X peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("c2", "c5"), default=os.environ.get("CRDT_BENCH_WORKLOAD", "c2"),
                    help="c2: GCounter+PNCounter 1M x 256 (BASELINE config 2) + a config-5 block; c5: VClock "
                         "1M x 1024 per GPU (one shard of config 5) only")
    ap.add_argument("--c5", action=argparse.BooleanOptionalAction, default=True,
                    help="with --workload c2: also time config 5's step and report it in the `c5` block")
    ap.add_argument("--replicas", type=int, default=R_REPLICAS, help="replicas per rank (configs 2 and 5: 1M)")
    ap.add_argument("--actors", type=int, default=None, help="default 256 (c2) / 1024 (c5)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="target fold seconds of the CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fused", action=argparse.BooleanOptionalAction, default=True,
                    help="all lubs of a step in one launch (crdt_lub_many_multi); --no-fused: one launch per lub")
    ap.add_argument("--exchange", choices=("cabi", "cabi-ops", "torch"), default="cabi",
                    help="N > 1: the C ABI over its own RCCL communicator, the C ABI over torch.distributed "
                         "host callbacks (crdt_ctx_comm_init_ops), or the torch.distributed twin")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm) for real runs; gloo lets several ranks share one GPU in tests")
    ap.add_argument("--c3", action=argparse.BooleanOptionalAction, default=None,
                    help="also time BASELINE config 3 (Orswot 65,536 x 4,096 x 64 with deferred removes) in a "
                         "`c3` block; default on at N = 1")
    ap.add_argument("--c4", action=argparse.BooleanOptionalAction, default=None,
                    help="also time BASELINE config 4 (Map<u32, MVReg<u64>> 16,384 x 1,024 x 32, V = 2) in a "
                         "`c4` block; default on at N = 1")
    ap.add_argument("--contig-input", action=argparse.BooleanOptionalAction, default=True,
                    help="generate each input batch in one physically contiguous device block (crdt_device_alloc) "
                         "when one is free")
    ap.add_argument("--causal-steps", type=int, default=5, help="timed lub_many calls of the c3 / c4 blocks")
    ap.add_argument("--parity-seed", type=int, default=1, help="member / key sample of the c3 / c4 parity checks")
    ap.add_argument("--parity-members", type=int, default=16)
    ap.add_argument("--parity-keys", type=int, default=16)
    ap.add_argument("--c3-cpu-replicas", type=int, default=1024, help="replicas of the c3 CPU baseline sample")
    ap.add_argument("--c4-cpu-replicas", type=int, default=4096, help="replicas of the c4 CPU baseline sample")
    ap.add_argument("--c3-cpu-replicas-per-thread", type=int, default=256,
                    help="replicas per host thread of the c3 multi-core CPU baseline")
    ap.add_argument("--c4-cpu-mt-replicas", type=int, default=8192,
                    help="replicas of the c4 multi-core CPU baseline (key ranges per thread)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="PMC-derived HBM bytes per launch (written by profiles/collect.sh)")
    return ap.parse_args()


KERNEL_SOURCES = {"c2": "lattice.hip", "c5": "lattice.hip", "c3": "orswot.hip", "c4": "map.hip"}


def kernel_source_sha(block="c2"):
    """sha256 of the source of a block's dominant kernel (c2 / c5: lub_multi_kernel /
    lub_stream_kernel, csrc/lattice.hip; c3: orswot_join_kernel, csrc/orswot.hip; c4:
    map_fold_kernel, csrc/map.hip): a PMC traffic figure is reported only for the kernel source it
    was measured on."""
    import hashlib
    with open(os.path.join(ROOT, "rust-crdt_amd", "csrc", KERNEL_SOURCES[block]), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic(args, block, workload):
    """(hbm bytes per launch, source note) from profiles/pmc_traffic.json — one entry per block,
    used only when the entry's workload and kernel source sha256 match this run."""
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, "not collected for this kernel source (profiles/collect.sh writes it)"
    e = tj.get(block) if isinstance(tj.get(block), dict) else None
    if e and e.get("workload") == workload and e.get("kernel_source_sha256") == kernel_source_sha(block):
        return e.get("hbm_bytes_per_launch"), (
            f"{e.get('source')}: rocprofv3 FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE per launch of "
            f"{e.get('kernel')}, separate --pmc passes, same kernel source (sha256 of csrc/{KERNEL_SOURCES[block]})")
    return None, "not collected for this kernel source (profiles/collect.sh writes it)"


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def self_launch(args):
    """--gpus N > 1 without a torchrun environment: start N ranks in a fresh child (this process has
    not touched the GPU) and relay its output and exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.run(cmd, env=env).returncode


def cpu_threads():
    """Host threads for the CPU baseline: the CPUs this process may run on, at most 16 (the
    GPU box's CPU share; os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(args, workload, actors):
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
            if workload == "c5":
                v = O.synth_matrix(SEED_V, n, actors, 0, row0=row0)
                _, tv = O.counter_fold_mt(v, False, threads)
                fold_s += tv
                done_rows += n
            else:
                g = O.synth_matrix(SEED_G, n, actors, 0, row0=row0)
                _, tg = O.counter_fold_mt(g, False, threads)
                p = O.synth_matrix(SEED_P, n, 2 * actors, 0, row0=row0)
                _, tp = O.counter_fold_mt(p, True, threads)
                fold_s += tg + tp
                done_rows += 2 * n
            reps += 1
        return done_rows / fold_s, reps, fold_s

    def run_dense(threads, rows_per_rep, seconds):
        """SURVEY §8d CPU timing (3): the same fold on the dense SoA rows (elementwise u64 max over
        row ranges per thread, oracle_dense_max_mt) — the CPU's own bandwidth roofline."""
        done_rows, fold_s, reps = 0, 0.0, 0
        m = O.synth_matrix(SEED_V if workload == "c5" else SEED_G, rows_per_rep, actors, 0)
        t_start = time.time()
        while fold_s < seconds and time.time() - t_start < 4 * seconds:
            _, t = O.dense_max_mt(m, threads)
            fold_s += t
            done_rows += rows_per_rep
            reps += 1
        return done_rows / fold_s, reps, fold_s, m.nbytes

    if workload == "c5":
        v1, reps1, s1 = run(1, 4096, args.cpu_seconds / 2)
        vT, repsT, sT = run(T, 2048, args.cpu_seconds)
        what = f"{repsT} x {T}x2048 VClock x {actors} replicas"
        one = f"{reps1} x 4096 replicas, {s1:.2f} s of fold"
    else:
        v1, reps1, s1 = run(1, 16384, args.cpu_seconds / 2)
        vT, repsT, sT = run(T, 4096, args.cpu_seconds)
        what = f"{repsT} x ({T}x4096 GCounter x {actors} + {T}x4096 PNCounter x 2x{actors}) replicas"
        one = f"{reps1} x (16384 + 16384) replicas, {s1:.2f} s of fold"
    vd, repsd, sd, nb = run_dense(T, 1 << 18, max(1.0, args.cpu_seconds / 4))
    return {
        "value": vT,
        "unit": "replica-merges/s",
        "cores": T,
        "kind": "port",
        "sample": (f"{what} of the same synthetic input, left fold of the restated VClock::merge over std::map "
                   f"(oracle/ref_fold.cpp) split over {T} threads (this job's CPU share of the GPU box) + final "
                   f"merge of the partials, map ingest excluded; {sT:.2f} s of fold"),
        "single_core": {"value": v1, "cores": 1, "sample": one},
        "dense_soa": {"value": vd, "cores": T, "GBs": vd * nb / (1 << 18) / 1e9,
                      "sample": (f"{repsd} x elementwise max over {1 << 18} dense rows x {actors} u64 "
                                 f"({nb / 2**20:.0f} MiB, {sd:.2f} s) split over {T} threads (oracle_dense_max_mt): "
                                 "the CPU fold without the reference's map containers")},
    }


class Env:
    """The ranks, the ctx and the chosen exchange."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        import crdts_gpu as cg
        from crdts_gpu import dist as cdist

        self.torch, self.dist, self.cg, self.cdist = torch, dist, cg, cdist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dev = local % torch.cuda.device_count()
        torch.cuda.set_device(self.dev)
        if self.world > 1:
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.dev))
            else:
                dist.init_process_group(args.dist_backend)
        self.ctx = cg.Context.default(self.dev)
        self.exchange = args.exchange if self.world > 1 else "none"
        self.cabi = self.world > 1 and args.exchange in ("cabi", "cabi-ops")
        self.note = ""
        if self.world > 1 and args.exchange == "cabi":
            uid = [cg.shard.unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            up = 1
            try:
                cg.shard.comm_init(self.ctx, uid[0], self.world, self.rank)
                self.note = cg.shard.comm_note(self.ctx)[0]
            except Exception as e:  # every rank learns it below and all take the torch exchange together
                print(f"rank {self.rank}: crdt_ctx_comm_init failed ({e}); using the torch.distributed exchange",
                      file=sys.stderr)
                up = 0
            # every rank must be up before any rank enters the probe (a collective): a rank whose init
            # failed would otherwise leave the others blocked in the probe's header all-gather
            flag = torch.tensor([up], dtype=torch.int64, device="cuda")
            cdist.all_reduce_(flag, dist.ReduceOp.MIN)
            up = int(flag.item())
            if up:  # one small C-ABI exchange before the real ones: the result must be the global max
                try:
                    probe = torch.full((4, 8), self.rank + 1, dtype=torch.int64, device="cuda")
                    got = cg.shard.lub_many_sharded("vclock", probe, ctx=self.ctx)
                    torch.cuda.synchronize()
                    if not bool((got == self.world).all()):
                        raise RuntimeError(f"probe exchange returned {got.tolist()}, expected {self.world}")
                except Exception as e:
                    print(f"rank {self.rank}: C-ABI probe exchange failed ({e}); using the torch.distributed "
                          "exchange", file=sys.stderr)
                    up = 0
            flag = torch.tensor([up], dtype=torch.int64, device="cuda")
            cdist.all_reduce_(flag, dist.ReduceOp.MIN)
            if not int(flag.item()):
                try:
                    cg.shard.comm_destroy(self.ctx)
                except Exception:
                    pass
                self.cabi = False
                self.exchange = "torch (C-ABI communicator setup or probe exchange failed)"
        elif self.world > 1 and args.exchange == "cabi-ops":
            cg.shard.comm_init_ops(self.ctx, cg.shard.TorchCommOps(), self.world, self.rank)

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, vals):
        t = self.torch.tensor(vals, dtype=self.torch.float64, device="cuda")
        if self.world > 1:
            self.cdist.all_reduce_(t, self.dist.ReduceOp.MAX)
        return t.tolist()


def oracle_parity_counters(args, torch, lubs, outs, A):
    """The oracle's restated GCounter / PNCounter / VClock fold (VClock::merge vclock.rs:130-136 over
    ordered maps, oracle_counter_fold_mt over the host's threads) on a sample of actors over EVERY
    replica row of the launch, against the same words of the GPU result (outside the timed region)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    t0 = time.time()
    acts = np.sort(np.random.default_rng(args.parity_seed).choice(A, size=min(args.parity_members, A),
                                                                   replace=False))
    ok, rows = True, 0
    for (kind, x, _), o in zip(lubs, outs):
        pn = kind == "pncounter"
        cols = np.concatenate([acts, acts + A]) if pn else acts
        idx = torch.from_numpy(cols.astype(np.int64)).to(x.device)
        sub = np.ascontiguousarray(x.index_select(1, idx).cpu().numpy().view(np.uint64))
        exp, _ = O.counter_fold_mt(sub, pn, cpu_threads())
        got = o.index_select(0, idx).cpu().numpy().view(np.uint64)
        ok = ok and bool(np.array_equal(exp, got))
        rows += sub.shape[0]
    return {"result": "ok" if ok else "MISMATCH",
            "sample": (f"{len(acts)} actors (seed {args.parity_seed}) x every replica row "
                       f"({rows} rows over {len(lubs)} lub(s)), oracle_counter_fold_mt on {cpu_threads()} threads"),
            "seconds": time.time() - t0}


def run_workload(args, env, workload):
    """Generate the rank's shard in HBM, warm up, time args.steps steps; return the measured block."""
    torch, cg, cdist = env.torch, env.cg, env.cdist
    ctx, world, rank = env.ctx, env.world, env.rank
    R = args.replicas
    A = args.actors if (args.actors is not None and workload == args.workload) else (A_C5 if workload == "c5" else A_ACTORS)
    # Synthetic replicas, generated in HBM; rank k owns rows [k*R, (k+1)*R) of the global input.
    def alloc(shape):  # one contiguous device block where one is free (--contig-input), else torch's
        t = ctx.device_empty(shape) if args.contig_input else None
        return t if t is not None else torch.empty(shape, dtype=torch.int64, device="cuda")

    if workload == "c5":
        lubs = [("vclock", alloc((R, A)), SEED_V)]
    else:
        lubs = [("gcounter", alloc((R, A)), SEED_G), ("pncounter", alloc((R, 2 * A)), SEED_P)]
    for _, x, seed in lubs:
        cg.synth_fill(ctx, x, seed, 0, first_row=rank * R)
    outs = [torch.empty((x.shape[1],), dtype=torch.int64, device="cuda") for _, x, _ in lubs]
    mods = {"vclock": cg.vclock, "gcounter": cg.gcounter, "pncounter": cg.pncounter}
    items = [(kind, x, o) for (kind, x, _), o in zip(lubs, outs)]
    fused = args.fused and len(lubs) > 1
    torch.cuda.synchronize()

    def step():
        if fused:  # every lub of the step in ONE launch (crdt_lub_many_multi)
            if env.cabi:  # + one grouped all-reduce MAX per step
                cg.shard.lub_many_multi_sharded(items, ctx=ctx)
            else:
                cg.lub_many_multi(items, ctx=ctx)
                if world > 1:
                    for o in outs:
                        cdist.allreduce_umax_(o)
            return
        for (kind, x, _), o in zip(lubs, outs):
            if env.cabi:  # local lub + one all-reduce MAX, one C call
                o.copy_(cg.shard.lub_many_sharded(kind, x, ctx=ctx))
            else:
                mods[kind].lub_many(x, out=o, ctx=ctx)
                if world > 1:  # torch.distributed twin: sign-biased MAX all-reduce
                    cdist.allreduce_umax_(o)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    env.barrier()
    ctx.timing_reset()
    ctx.set_timing(True)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    env.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    kern_ms, launches = ctx.timing("lub_stream")
    xch_ms, xch_n = ctx.timing("shard_exchange")  # C-ABI exchange collectives (HIP events, ctx stream)
    agr_ms, agr_n = ctx.timing("shard_agree")     # C-ABI header agreement (host wall time per call)
    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    step_ms = env.max_over_ranks(step_ms)
    elapsed = env.max_over_ranks([elapsed])[0]
    xch_ms, agr_ms = env.max_over_ranks([xch_ms, agr_ms])

    # Parity (outside the timed region): unsigned max with torch ops; for N > 1 the exchanged
    # result must equal the max over every rank's torch reference (torch.distributed's own exchange)
    sign = torch.tensor(-(2**63), dtype=torch.int64, device="cuda")
    refs = [(x ^ sign).amax(0) ^ sign for _, x, _ in lubs]
    got, ref = torch.cat(outs), torch.cat(refs)
    if world > 1:
        cdist.allreduce_umax_(ref)
    ok = env.max_over_ranks([0.0 if bool(torch.equal(got, ref)) else 1.0])[0] == 0.0
    # and (N = 1, rank 0, with the CPU leg) the oracle's restated fold on a sample of actors over
    # every replica row: the CPU check the c3 / c4 blocks already carry
    oracle_par = {"result": "unchecked (the oracle leg runs at N = 1 without --no-cpu-baseline)"}
    if world == 1 and not args.no_cpu_baseline:
        oracle_par = oracle_parity_counters(args, torch, lubs, outs, A)

    merges_per_step = len(lubs) * R * world
    bytes_per_step = sum(R * x.shape[1] * 8 + x.shape[1] * 8 for _, x, _ in lubs)
    launches_per_step = launches / args.steps if launches else float(len(lubs))
    avg_launch_bytes = bytes_per_step / launches_per_step
    avg_launch_s = (kern_ms / 1e3) / launches if launches else float("nan")
    achieved = avg_launch_bytes / avg_launch_s / 1e9
    srt = sorted(step_ms)
    med = srt[len(srt) // 2] if len(srt) % 2 else 0.5 * (srt[len(srt) // 2 - 1] + srt[len(srt) // 2])
    name = (f"vclock lub {R}x{A} (config 5 shard)" if workload == "c5" else f"gcounter+pncounter lub {R}x{A}")
    traffic, traffic_src = pmc_traffic(args, workload, name)
    if workload == "c2" and not fused:
        traffic, traffic_src = None, "collected for the fused launch only"
    if env.cabi:
        exch = ((f"C-ABI crdt_lub_many_multi_sharded: one grouped all-reduce MAX " if fused
                 else "C-ABI crdt_*_lub_many_sharded: all-reduce MAX ")
                + f"of the partial lubs ({sum(x.shape[1] for _, x, _ in lubs)} u64 words per step) over "
                + ("the ctx's RCCL communicator (ncclUint64, ncclMax)" if args.exchange == "cabi"
                   else "crdt_ctx_comm_init_ops host callbacks (torch.distributed " + args.dist_backend + ")"))
    elif world > 1:
        exch = f"torch.distributed all-reduce MAX (sign-biased u64); --exchange {env.exchange}"
    else:
        exch = "none"
    block = {
        "value": merges_per_step * args.steps / elapsed,
        "unit": "replica-merges/s",
        "ms_per_step": elapsed / args.steps * 1e3,
        "step_ms": {"median": med, "min": srt[0], "max": srt[-1], "source": "HIP events around each step, "
                    "max over ranks"},
        "config": {
            "workload": name,
            "replicas_per_gpu": R,
            "actors": A,
            "types": (["VClock (A u64)"] if workload == "c5" else ["GCounter (A u64)", "PNCounter (2A u64)"]),
            "replica_merges_per_step": merges_per_step,
            "exchange": exch,
            "parallelism": f"replica-shard x{world}",
            "launches_per_step": launches_per_step,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": (("lub_multi_kernel<Max,2,8>" if fused else "lub_stream_kernel<Max,2,8>")
                       + (" (VClock launch)" if workload == "c5" else
                          (" (GCounter + PNCounter in one launch)" if fused else " (GCounter + PNCounter launches)"))),
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "avg_launch_us": avg_launch_s * 1e6,
            "launches": launches,
            "algorithmic_bytes_per_launch": avg_launch_bytes,
        },
        "parity": "ok" if ok and oracle_par["result"] != "MISMATCH" else "MISMATCH",
        "parity_detail": {"torch_umax": "ok" if ok else "MISMATCH", "oracle": oracle_par},
    }
    if env.cabi:  # where a scaling loss goes: the exchange collectives and the per-call agreement
        block["exchange"] = {
            "exchange_ms_per_step": xch_ms / args.steps, "exchange_calls": xch_n,
            "agree_ms_per_step": agr_ms / args.steps, "agree_calls": agr_n,
            "source": "libcrdt_gpu timers, max over ranks: shard_exchange = HIP events around the exchange "
                      "collectives on the ctx stream; shard_agree = host wall time of the validation-header "
                      "all-gather of each sharded call (csrc/shard.hip)"}
    del lubs, outs, items
    torch.cuda.empty_cache()
    return block, A


C3 = dict(R=65536, M=4096, A=64, kmax=48, p_def=0.1, seed=0x5EED0003)
C4 = dict(R=16384, K=1024, A=32, V=2, kmax=256, p_def=0.1, seed=0x5EED0004, vout=4)


def c3_oracle_leg(args, inp, res, ctx):
    """BASELINE config 3 through the oracle (the checker; rank 0, N = 1 only).

    parity   the oracle's dense Orswot fold (join fold, then every deferred remove; cross-checked
             against the map-based restatement in tests/test_oracle_twins.py) over EVERY replica
             restricted to a member sample — the merge is independent per member given the clocks
             (orswot.rs:81-149) — plus every surviving deferred remove with its whole member set.
    baseline the map-based restatement of Orswot::merge (oracle/ref_fold.cpp, orswot.rs:81-149)
             folding the first replicas of the same HBM input with all members, one thread."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    u64 = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731
    R, M, A = C3["R"], C3["M"], C3["A"]
    msub = np.sort(np.random.default_rng(args.parity_seed).choice(M, size=args.parity_members, replace=False))
    tsub = torch.from_numpy(msub).cuda()
    clock_h, ent_h = u64(inp.clock), u64(inp.entries[:, tsub, :].contiguous())
    dcl_h, dmem_h = u64(inp.def_clock), u64(inp.def_members)
    got_c, got_e = u64(res.clock), u64(res.entries[tsub])
    keep, gmem = res.def_keep.cpu().numpy(), u64(res.def_members)
    D = dcl_h.shape[0]
    sub_mem = np.zeros((D, (len(msub) + 63) // 64), np.uint64)
    for j, m in enumerate(msub):
        sub_mem[:, j // 64] |= ((dmem_h[:, m // 64] >> np.uint64(m % 64)) & np.uint64(1)) << np.uint64(j % 64)
    t0 = time.time()
    oc, oe, _ = O.dense_orswot_lub(clock_h, ent_h, dcl_h, sub_mem)
    exp_def = O.dense_orswot_survivors(oc, dcl_h, dmem_h)
    got_def = {(tuple(int(x) for x in dcl_h[d]), O.bitmap_members(gmem[d])) for d in np.flatnonzero(keep)}
    ok = bool(np.array_equal(got_c, oc) and np.array_equal(got_e, oe) and got_def == exp_def)
    check_s = time.time() - t0
    parity = {"result": "ok" if ok else "MISMATCH",
              "method": (f"oracle dense Orswot fold over all {R} replicas on {len(msub)} sampled members (seed "
                         f"{args.parity_seed}) + all {len(exp_def)} surviving deferred removes with whole member "
                         f"sets ({D} removes in the input)"), "check_s": check_s}
    # CPU baseline: the map-based fold of the first Rc replicas (all members), their own removes
    Rc = min(R, args.c3_cpu_replicas)
    off = np.asarray(inp.def_off, np.int64)  # per-replica CSR offsets (R + 1) of the generator
    dend = int(off[Rc])
    c_h = u64(inp.clock[:Rc])
    e_h = u64(inp.entries[:Rc])
    d_off = off[:Rc + 1].astype(np.uint64)
    _, _, _, fold_s = O.orswot_fold(c_h, e_h, d_off, dcl_h[:dend], dmem_h[:dend])
    del e_h
    one = {"value": Rc / fold_s, "unit": "replica-merges/s", "cores": 1, "kind": "port",
           "sample": (f"first {Rc} of the {R} replicas (all {M} members x {A} actors, their {dend} deferred "
                      f"removes), left fold of the restated Orswot::merge over std::unordered_map / std::map "
                      f"states (oracle/ref_fold.cpp), 1 thread, ingest excluded; {fold_s:.2f} s of fold")}
    # the same fold over the host's threads (SURVEY §8d CPU timing (2)): replica ranges per thread, the
    # partial states merged in order (oracle_orswot_fold_mt; tests/test_oracle_mt.py: same result)
    T = cpu_threads()
    Rm = min(R, args.c3_cpu_replicas_per_thread * T)
    dm = int(off[Rm])
    e_h = u64(inp.entries[:Rm])
    _, _, _, mt_s = O.orswot_fold(u64(inp.clock[:Rm]), e_h, off[:Rm + 1].astype(np.uint64), dcl_h[:dm], dmem_h[:dm],
                                  threads=T)
    del e_h
    base = {"value": Rm / mt_s, "unit": "replica-merges/s", "cores": T, "kind": "port",
            "sample": (f"subsample: first {Rm} of the {R} replicas (all {M} members x {A} actors, their {dm} deferred "
                       f"removes), the restated Orswot::merge over std::unordered_map / std::map states "
                       f"(oracle/ref_fold.cpp oracle_orswot_fold_mt) split over {T} threads by replica ranges + the "
                       f"final merge of the {T} partial states, ingest excluded; {mt_s:.2f} s of fold"),
            "single_core": one}
    return parity, base


def c4_oracle_leg(args, inp, res, ctx):
    """BASELINE config 4 through the oracle (the checker; rank 0, N = 1 only).

    parity   the restated Map::merge fold over map-based states (oracle/ref_fold.cpp,
             map.rs:140-220) over EVERY replica restricted to a key sample (keys are independent
             given the replica clocks and the deferred list), plus the surviving removes restricted
             to the sample.
    baseline the same restated fold over the first replicas with all keys, one thread."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    u64 = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731
    R, K, A, V, vout = C4["R"], C4["K"], C4["A"], C4["V"], C4["vout"]
    keys = np.sort(np.random.default_rng(args.parity_seed).choice(K, size=args.parity_keys, replace=False))
    tk = torch.from_numpy(keys).cuda()
    clock_h = u64(inp.clock)
    ec_h, vc_h, vv_h = (u64(t[:, tk].contiguous()) for t in (inp.ec, inp.vclk, inp.vval))
    rows = inp.def_row.cpu().numpy().astype(np.int64)
    dcl_h, dks_h = u64(inp.def_clock), u64(inp.def_keys)
    t0 = time.time()
    exp = O.map_fold(clock_h, ec_h, vc_h, vv_h, rows, dcl_h, O.restrict_deferred_keys(dks_h, keys), vout)
    ok = (np.array_equal(u64(res.clock), exp[0]) and np.array_equal(u64(res.ec)[keys], exp[1])
          and np.array_equal(u64(res.vclk)[keys], exp[2]) and np.array_equal(u64(res.vval)[keys], exp[3])
          and np.array_equal(res.nval.cpu().numpy()[keys], exp[4]) and int(res.flags.max()) == 0)
    pos = {int(k): i for i, k in enumerate(keys)}
    gk = u64(res.def_keys)
    got_sub = set()
    for j in np.flatnonzero(res.def_keep.cpu().numpy()):
        s = frozenset(pos[k] for k in O.bitmap_members(gk[j]) if k in pos)
        if s:
            got_sub.add((tuple(int(x) for x in dcl_h[j]), s))
    ok = bool(ok and got_sub == {x for x in exp[5] if x[1]})
    parity = {"result": "ok" if ok else "MISMATCH",
              "method": (f"restated Map::merge fold (oracle/ref_fold.cpp) over all {R} replicas on {len(keys)} "
                         f"sampled keys (seed {args.parity_seed}), incl. the surviving removes restricted to them"),
              "check_s": time.time() - t0}
    Rc = min(R, args.c4_cpu_replicas)
    sel = rows < Rc
    e_h = [u64(t[:Rc]) for t in (inp.clock, inp.ec, inp.vclk, inp.vval)]
    fold_s = O.map_fold(*e_h, rows[sel], dcl_h[sel], dks_h[sel], vout)[6]
    del e_h
    one = {"value": Rc / fold_s, "unit": "replica-merges/s", "cores": 1, "kind": "port",
           "sample": (f"first {Rc} of the {R} replicas (all {K} keys, {int(sel.sum())} deferred removes), left "
                      f"fold of the restated Map::merge over std::map states (oracle/ref_fold.cpp), 1 thread, "
                      f"ingest excluded; {fold_s:.2f} s of fold")}
    # the same fold over the host's threads: KEY ranges per thread over every replica of the sample (the
    # Map fold is not associative, so not replica ranges; keys are independent given the clocks and the
    # removes — oracle_map_fold_mt, tests/test_oracle_mt.py: same result)
    T = cpu_threads()
    Rm = min(R, args.c4_cpu_mt_replicas)
    sel = rows < Rm
    e_h = [u64(t[:Rm]) for t in (inp.clock, inp.ec, inp.vclk, inp.vval)]
    mt_s = O.map_fold(*e_h, rows[sel], dcl_h[sel], dks_h[sel], vout, threads=T)[6]
    del e_h
    base = {"value": Rm / mt_s, "unit": "replica-merges/s", "cores": T, "kind": "port",
            "sample": (f"subsample: first {Rm} of the {R} replicas (all {K} keys, {int(sel.sum())} deferred removes), "
                       f"the restated Map::merge left fold over std::map states (oracle/ref_fold.cpp "
                       f"oracle_map_fold_mt) split over {T} threads by key ranges, ingest excluded; {mt_s:.2f} s of fold"),
            "single_core": one}
    return parity, base


def run_causal(args, env, block):
    """BASELINE config 3 (Orswot) or 4 (Map<u32, MVReg<u64>>) at full size on this GPU: generate the
    replicas in HBM, time args.steps lub_many calls (one step = one fold of every replica), report
    the dominant kernel's roofline, and (rank 0, N = 1) the oracle's parity check and CPU baseline."""
    torch, cg = env.torch, env.cg
    from crdts_gpu import synth
    ctx = env.ctx
    if block == "c3":
        p = C3
        # the 128 GiB of replicas in one physically contiguous block where one is free (fewer
        # translation misses for the one streaming pass), else the torch allocator
        ent = ctx.device_empty((p["R"], p["M"], p["A"])) if args.contig_input else None
        alloc = "contiguous block (crdt_device_alloc)" if ent is not None else "torch caching allocator"
        inp = synth.orswot_replicas(ctx, p["R"], p["M"], p["A"], seed=p["seed"], kmax=p["kmax"], p_def=p["p_def"],
                                    entries=ent)
        D = inp.def_clock.shape[0]
        goff = [0, D]

        def step():
            return cg.orswot.lub_many(inp.clock, inp.entries, def_off=goff, def_clock=inp.def_clock,
                                      def_members=inp.def_members, ctx=ctx)
        R = p["R"]
        name = f"orswot<u64,u32> lub {R}x{p['M']}x{p['A']} (config 3)"
        timer, kernel = "orswot_join", "orswot_join_kernel"
        alg = (R + 1) * (p["M"] * p["A"] + p["A"]) * 8
        alg_note = "8·(M·A + A) per replica read + the (M·A + A) u64 output"
        cfg = {"replicas": R, "members": p["M"], "actors": p["A"], "deferred_removes": D,
               "types": ["Orswot<u64 member, u32 actor>"], "input_alloc": alloc}
    else:
        p = C4
        inp = synth.map_replicas(ctx, p["R"], p["K"], p["A"], p["V"], p["seed"], kmax=p["kmax"], p_def=p["p_def"],
                                 contig=args.contig_input)
        D = inp.def_clock.shape[0]

        def step():
            return cg.map.lub_many(inp.clock, inp.ec, inp.vclk, inp.vval, def_off=inp.def_off,
                                   def_row=inp.def_row, def_clock=inp.def_clock, def_keys=inp.def_keys,
                                   vout=p["vout"], ctx=ctx, check=False)
        R, K, A, V, vout = p["R"], p["K"], p["A"], p["V"], p["vout"]
        Kw = (K + 63) // 64
        name = f"map<u32,mvreg<u64>> lub {R}x{K}x{A} V={V} (config 4)"
        timer, kernel = "map_fold", "map_fold_kernel"
        alg = (R * (K * (A * 8 + V * A * 8 + V * 8) + A * 8) + D * (A + Kw + 1) * 8
               + K * (A + vout * A + vout) * 8 + A * 8)
        alg_note = ("8·(K·(A + V·A + V) + A) per replica read + 8·(A + Kw + 1) per deferred remove + the "
                    "K·(A + Vout·A + Vout) + A u64 output")
        cfg = {"replicas": R, "keys": K, "actors": A, "value_slots": V, "deferred_removes": D,
               "types": ["Map<u32, MVReg<u64>>"], "input_alloc": inp.alloc}
    torch.cuda.synchronize()
    res = None
    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    env.barrier()
    ctx.timing_reset()
    ctx.set_timing(True)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.causal_steps + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    for i in range(args.causal_steps):
        res = step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    env.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    kern_ms, launches = ctx.timing(timer)
    step_ms = env.max_over_ranks([evs[i].elapsed_time(evs[i + 1]) for i in range(args.causal_steps)])
    elapsed = env.max_over_ranks([elapsed])[0]
    srt = sorted(step_ms)
    avg_launch_s = (kern_ms / 1e3) / launches if launches else float("nan")
    achieved = alg / avg_launch_s / 1e9
    traffic, traffic_src = pmc_traffic(args, block, name)
    block_out = {
        "metric": METRIC + (" — BASELINE config 3 (Orswot)" if block == "c3" else " — BASELINE config 4 (Map)"),
        "value": R * env.world * args.causal_steps / elapsed,
        "unit": "replica-merges/s",
        "steps": args.causal_steps,
        "ms_per_step": elapsed / args.causal_steps * 1e3,
        "step_ms": {"median": srt[len(srt) // 2], "min": srt[0], "max": srt[-1],
                    "source": "HIP events around each lub_many (all of its kernels), max over ranks"},
        "config": dict(cfg, workload=name, parallelism="one GPU (replicas in HBM)"),
        "roofline": {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "avg_launch_us": avg_launch_s * 1e6, "launches": launches,
                     "algorithmic_bytes_per_launch": alg, "algorithmic_bytes_rule": alg_note},
        "parity": {"result": "unchecked (the oracle leg runs at N = 1 without --no-cpu-baseline)"},
        "cpu_baseline": None,
    }
    if env.world == 1 and env.rank == 0 and not args.no_cpu_baseline:
        leg = c3_oracle_leg if block == "c3" else c4_oracle_leg
        block_out["parity"], block_out["cpu_baseline"] = leg(args, inp, res, ctx)
    del inp, res
    torch.cuda.empty_cache()
    return block_out


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        sys.exit(self_launch(args))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to time a different world "
              "size than requested", file=sys.stderr)
        sys.exit(2)
    env = Env(args)
    head, A = run_workload(args, env, args.workload)
    c5 = None
    if args.workload == "c2" and args.c5:
        c5, _ = run_workload(args, env, "c5")
    causal = {}
    for blk in ("c3", "c4"):
        on = getattr(args, blk)
        if on is None:
            on = env.world == 1
        if on:
            causal[blk] = run_causal(args, env, blk)
    ok = (head["parity"] == "ok" and (c5 is None or c5["parity"] == "ok")
          and all(b["parity"]["result"] != "MISMATCH" for b in causal.values()))
    if env.rank == 0:
        out = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "replica-merges/s",
            "n_gpus": env.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "step_ms": head["step_ms"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (counter-based splitmix64 replicas generated in HBM, seeds 0x5EED0002/3/5)",
            "config": head["config"],
            "roofline": head["roofline"],
            "cpu_baseline": None,
            "parity": head["parity"],
            "parity_detail": head["parity_detail"],
        }
        if "exchange" in head:
            out["exchange"] = head["exchange"]
        if env.note:
            out["config"]["rccl_note"] = env.note
        if c5 is not None:
            out["c5"] = dict(c5, metric=METRIC + " — BASELINE config 5 (VClock 1,024 actors; 8M replicas at 8 GPUs)")
        out.update(causal)
        if env.world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, args.workload, A)
        print(json.dumps(out), flush=True)
    if env.world > 1:
        if env.cabi:
            env.cg.shard.comm_destroy(env.ctx)
        env.dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
