"""End-to-end merge of serialized replicas on one MI355X: the states arrive as
serde / bincode 1.x frames in host memory, and a batch lub is
    H2D of the frames (pinned) -> crdt_*_ingest -> crdt_*_lub_many -> crdt_*_egress -> D2H,
next to the device-resident lub alone.  Workloads: config 2 (GCounter and PNCounter, 1M replicas x
256 actors) and a config-3 Orswot slice (R replicas x 4,096 members x 64 actors, u64 members).

The input frames are produced by the device egress of synthetic dense states (byte-exact against
the oracle's bincode restatement in tests/test_gpu_wire.py); every run checks ingest(frames) ==
the dense states and the merged result against torch (counters) / a re-ingest round trip (Orswot).
Prints one JSON line per workload."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-crdt_amd"))

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import synth, wire  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=1 << 20)
ap.add_argument("--actors", type=int, default=256)
ap.add_argument("--orswot-replicas", type=int, default=4096)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--map-replicas", type=int, default=4096)
ap.add_argument("--skip", default="", help="comma list of workloads to skip: gcounter,pncounter,orswot,map")
args = ap.parse_args()
skip = set(args.skip.split(",")) if args.skip else set()

torch.cuda.set_device(0)
ctx = cg.Context(0)
dev = torch.device("cuda", 0)


def ev_time(fn, steps):
    """Average ms of fn() over `steps` runs by HIP events on torch's current stream (the ctx's
    default stream is the null stream torch also uses here)."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def counters(kind):
    R, A = args.replicas, args.actors
    W = 2 * A if kind == "pncounter" else A
    rows = torch.empty((R, W), dtype=torch.int64, device=dev)
    cg.synth_fill(ctx, rows, 0x5EED0002 if kind == "gcounter" else 0x5EED0003, 0)
    actors = torch.arange(1, A + 1, dtype=torch.int32, device=dev) * 7  # sorted u32 actor ids
    ingest = wire.vclock_ingest if kind == "gcounter" else wire.pncounter_ingest
    egress = wire.vclock_egress if kind == "gcounter" else wire.pncounter_egress
    mod = cg.gcounter if kind == "gcounter" else cg.pncounter
    t0 = time.perf_counter()
    off, frames = egress(rows, actors, ctx=ctx)
    torch.cuda.synchronize()
    nbytes = frames.numel()
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    host.copy_(frames)
    host_off = off.cpu()
    setup_s = time.perf_counter() - t0
    # parity: ingest reproduces the dense states exactly
    back, st = ingest(frames, off, actors, ctx=ctx)
    ok = bool(torch.equal(back, rows)) and int(st.abs().sum()) == 0
    dense_out = torch.empty((W,), dtype=torch.int64, device=dev)
    ms_lub = ev_time(lambda: mod.lub_many(rows, out=dense_out, ctx=ctx), args.steps)
    ms_ing = ev_time(lambda: ingest(frames, off, actors, out=back, ctx=ctx), args.steps)
    ms_egr = ev_time(lambda: egress(rows[:65536], actors, ctx=ctx), args.steps)
    dframes = torch.empty_like(frames)
    doff = torch.empty_like(off)

    def e2e():
        dframes.copy_(host, non_blocking=True)
        doff.copy_(host_off, non_blocking=True)
        dense, _ = ingest(dframes, doff, actors, out=back, ctx=ctx)
        lub = mod.lub_many(dense, out=dense_out, ctx=ctx)
        o2, f2 = egress(lub[None], actors, ctx=ctx)
        return f2.cpu()

    e2e()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        res = e2e()
    ms_e2e = (time.perf_counter() - t1) / args.steps * 1e3
    sign = torch.tensor(-(2**63), dtype=torch.int64, device=dev)
    ref = (rows ^ sign).amax(0) ^ sign
    got, _ = ingest(res.to(dev), torch.tensor([0, res.numel()], dtype=torch.int64, device=dev), actors, ctx=ctx)
    ok = ok and bool(torch.equal(got[0], ref))
    ms_h2d = ev_time(lambda: dframes.copy_(host, non_blocking=True), 2)
    print(json.dumps({
        "workload": f"{kind} {R}x{A} from bincode frames", "frames_bytes": nbytes, "dense_bytes": R * W * 8,
        "ingest_ms": ms_ing, "ingest_GBs_frames": nbytes / ms_ing / 1e6,
        "ingest_GBs_frames_plus_dense": (nbytes + R * W * 8) / ms_ing / 1e6,
        "egress_ms_65536_rows": ms_egr, "lub_ms_device_resident": ms_lub,
        "h2d_ms": ms_h2d, "h2d_GBs": nbytes / ms_h2d / 1e6,
        "end_to_end_ms": ms_e2e, "end_to_end_replica_merges_per_s": R / ms_e2e * 1e3,
        "device_resident_replica_merges_per_s": R / ms_lub * 1e3,
        "setup_s": setup_s, "parity": "ok" if ok else "MISMATCH"}), flush=True)
    del rows, back, frames, dframes, host
    torch.cuda.empty_cache()
    return ok


def orswot():
    R, M, A = args.orswot_replicas, 4096, 64
    inp = synth.orswot_replicas(ctx, R, M, A, seed=0x5EED0003, kmax=48, p_def=0.1)
    D = inp.def_clock.shape[0]
    def_off = torch.from_numpy(inp.def_off.astype(np.int64)).to(dev)
    actors = torch.arange(1, A + 1, dtype=torch.int32, device=dev) * 3
    members = torch.arange(1, M + 1, dtype=torch.int64, device=dev) * 1000003
    off, frames = wire.orswot_egress(inp.clock, inp.entries, actors, members, def_off, inp.def_clock, inp.def_members,
                                     ctx=ctx)
    nbytes = frames.numel()
    res = wire.orswot_ingest(frames, off, actors, members, ctx=ctx)
    ok = (bool(torch.equal(res.clock, inp.clock)) and bool(torch.equal(res.entries, inp.entries))
          and bool(torch.equal(res.def_off, def_off)) and bool(torch.equal(res.def_clock, inp.def_clock))
          and bool(torch.equal(res.def_members, inp.def_members)) and int(res.status.abs().sum()) == 0)
    ms_ing = ev_time(lambda: wire.orswot_ingest(frames, off, actors, members, def_cap=D, ctx=ctx), args.steps)
    ms_egr = ev_time(lambda: wire.orswot_egress(inp.clock, inp.entries, actors, members, def_off, inp.def_clock,
                                                inp.def_members, ctx=ctx), max(1, args.steps // 2))
    ms_lub = ev_time(lambda: cg.orswot.lub_many(inp.clock, inp.entries, def_off=[0, D], def_clock=inp.def_clock,
                                                def_members=inp.def_members, ctx=ctx), args.steps)
    dense = R * M * A * 8 + R * A * 8
    print(json.dumps({
        "workload": f"orswot {R}x{M}x{A} (+{D} deferred) from bincode frames", "frames_bytes": nbytes,
        "dense_bytes": dense, "ingest_ms": ms_ing, "ingest_GBs_frames": nbytes / ms_ing / 1e6,
        "ingest_GBs_frames_plus_dense": (nbytes + 2 * dense) / ms_ing / 1e6,
        "egress_ms": ms_egr, "egress_GBs_frames": nbytes / ms_egr / 1e6, "lub_ms_device_resident": ms_lub,
        "parity": "ok" if ok else "MISMATCH"}), flush=True)
    return ok


def mapw():
    """Config-4-shaped Map<u32, MVReg<u64>> states (R x 1,024 keys x 32 actors, V = 2, deferred
    slots) -> egress -> frames -> ingest; ingest / egress GB/s of frames."""
    R, K, A, V = args.map_replicas, 1024, 32, 2
    inp = synth.map_replicas(ctx, R, K, A, V, 0x5EED0004, kmax=256, p_def=0.2)
    rows = inp.def_row.cpu().numpy().astype(np.int64)
    cnt = np.bincount(rows, minlength=R).astype(np.int32)
    Dcap = max(1, int(cnt.max()))
    Kw = (K + 63) // 64
    dcl = torch.zeros((R, Dcap, A), dtype=torch.int64, device=dev)
    dks = torch.zeros((R, Dcap, Kw), dtype=torch.int64, device=dev)
    slot = np.arange(rows.shape[0]) - np.searchsorted(rows, rows)
    rt, st_ = torch.from_numpy(rows).to(dev), torch.from_numpy(slot).to(dev)
    dcl[rt, st_] = inp.def_clock
    dks[rt, st_] = inp.def_keys
    states = cg.map.MapStates(inp.clock, inp.ec, inp.vclk, inp.vval, dcl, dks, torch.from_numpy(cnt).to(dev))
    actors = torch.arange(1, A + 1, dtype=torch.int32, device=dev) * 5
    keys = torch.arange(1, K + 1, dtype=torch.int32, device=dev) * 11
    off, frames = wire.map_egress(states, actors, keys, ctx=ctx)
    nbytes = frames.numel()
    back, status = wire.map_ingest(frames, off, actors, keys, V, Dcap, ctx=ctx)
    ok = int(status.abs().sum()) == 0 and all(bool(torch.equal(getattr(back, f), getattr(states, f)))
                                               for f in states._fields)
    ms_ing = ev_time(lambda: wire.map_ingest(frames, off, actors, keys, V, Dcap, ctx=ctx), args.steps)
    ms_egr = ev_time(lambda: wire.map_egress(states, actors, keys, ctx=ctx), max(1, args.steps // 2))
    dense = sum(t.numel() * 8 for t in (inp.clock, inp.ec, inp.vclk, inp.vval))
    print(json.dumps({
        "workload": f"map<u32,mvreg<u64>> {R}x{K}x{A} V={V} (+{int(cnt.sum())} deferred) from bincode frames",
        "frames_bytes": nbytes, "dense_bytes": dense, "ingest_ms": ms_ing, "ingest_GBs_frames": nbytes / ms_ing / 1e6,
        "ingest_GBs_frames_plus_dense": (nbytes + dense) / ms_ing / 1e6, "egress_ms": ms_egr,
        "egress_GBs_frames": nbytes / ms_egr / 1e6, "parity": "ok" if ok else "MISMATCH"}), flush=True)
    return ok


good = True
for k in ("gcounter", "pncounter"):
    if k not in skip:
        good = counters(k) and good
if "orswot" not in skip:
    good = orswot() and good
if "map" not in skip:
    torch.cuda.empty_cache()
    good = mapw() and good
sys.exit(0 if good else 3)
