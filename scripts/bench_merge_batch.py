"""In-place pairwise merge_batch of the causal types on one MI355X (crdt_orswot_merge_batch,
crdt_map_merge_batch): N independent self[i].merge(other[i]) over HBM-resident synthetic states
of the config-3 / config-4 shapes, HIP-event kernel time, algorithmic bytes (read self, read
other, write self) against 8 TB/s, and parity on sampled pairs against the oracle's one-pair
merge (Orswot::merge orswot.rs:81-149, Map::merge map.rs:140-220).  One JSON line per type."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-crdt_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--orswot-pairs", type=int, default=8192)
ap.add_argument("--map-pairs", type=int, default=8192)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--sample", type=int, default=4)
ap.add_argument("--contig", action="store_true", help="map: the states in contiguous device blocks")
ap.add_argument("--only", default="calib,orswot,map", help="comma list of: calib, orswot, map")
args = ap.parse_args()
torch.cuda.set_device(0)
ctx = cg.Context(0)
dev = torch.device("cuda", 0)
u64 = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731


def slots(def_off, def_clock, def_bits, N, Dcap):
    """Pooled removes (CSR by state) -> per-state slots (N, Dcap, .), counts."""
    off = np.asarray(def_off, np.int64)
    cnt = np.minimum(np.diff(off), Dcap).astype(np.int32)
    idx_s = np.repeat(np.arange(N), np.diff(off))
    idx_d = np.arange(off[-1]) - off[idx_s]
    keep = idx_d < Dcap
    A, Bw = def_clock.shape[1], def_bits.shape[1]
    dc = torch.zeros((N, Dcap, A), dtype=torch.int64, device=dev)
    db = torch.zeros((N, Dcap, Bw), dtype=torch.int64, device=dev)
    s_t, d_t = torch.from_numpy(idx_s[keep]).to(dev), torch.from_numpy(idx_d[keep]).to(dev)
    kt = torch.from_numpy(np.flatnonzero(keep)).to(dev)
    dc[s_t, d_t] = def_clock[kt]
    db[s_t, d_t] = def_bits[kt]
    return dc, db, torch.from_numpy(cnt).to(dev)


SPREAD = {}  # min / max of the last timed() call's steps (placement spread), library kernel times


def timed(fn, reset, kernel=None):
    reset()
    fn()
    torch.cuda.synchronize()
    ms = []
    ctx.timing_reset()
    for _ in range(args.steps):
        reset()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ctx.set_timing(kernel is not None)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ctx.set_timing(False)
        ms.append(s.elapsed_time(e))
    SPREAD.clear()
    SPREAD.update(ms_min=float(np.min(ms)), ms_max=float(np.max(ms)))
    if kernel:
        kms, n = ctx.timing(kernel)
        if n:
            SPREAD[kernel + "_ms"] = kms / n
    return float(np.median(ms))


def orswot():
    import oracle as O
    from orswot_apply_util import to_object
    N, M, A, Dcap = args.orswot_pairs, 4096, 64, 8
    a = synth.orswot_replicas(ctx, N, M, A, seed=0x5EED0003, kmax=48, p_def=0.2)
    b = synth.orswot_replicas(ctx, N, M, A, seed=0x5EED0003, kmax=48, first_row=N, p_def=0.2)
    sa = cg.orswot.OrswotStates(a.clock, a.entries, *slots(a.def_off, a.def_clock, a.def_members, N, 2 * Dcap))
    sb = cg.orswot.OrswotStates(b.clock, b.entries, *slots(b.def_off, b.def_clock, b.def_members, N, Dcap))
    keep = list(sa)
    work = cg.orswot.OrswotStates(*[x.clone() for x in sa])

    def reset():
        for d, s in zip(work, keep):
            d.copy_(s)

    ms = timed(lambda: cg.orswot.merge_batch(work, sb, ctx=ctx), reset)
    reset()
    status = cg.orswot.merge_batch(work, sb, ctx=ctx).cpu().numpy()
    ok = bool((status == 0).all())
    rng = np.random.default_rng(1)
    for i in rng.choice(N, size=args.sample, replace=False):
        i = int(i)
        ob = [to_object(u64(t[i:i + 1]), u64(e[i:i + 1]), u64(dc[i:i + 1]), u64(dm[i:i + 1]), n[i:i + 1].cpu().numpy(), 0)
              for t, e, dc, dm, n in (tuple(keep), tuple(sb))]
        exp = ob[0].copy()
        exp.merge(ob[1].copy())
        got = to_object(u64(work.clock[i:i + 1]), u64(work.entries[i:i + 1]), u64(work.def_clock[i:i + 1]),
                        u64(work.def_members[i:i + 1]), work.def_count[i:i + 1].cpu().numpy(), 0)
        ok = ok and got == exp
    alg = N * 3 * M * A * 8
    print(json.dumps({"op": "orswot_merge_batch", "pairs": N, "members": M, "actors": A, "kernel_ms_incl_deferred": ms,
                      "algorithmic_bytes": alg, "GBs": alg / ms / 1e6, "frac_of_8TBs": alg / ms / 8e9,
                      "pair_merges_per_s": N / ms * 1e3, "parity": "ok" if ok else "MISMATCH",
                      "parity_pairs": args.sample}), flush=True)
    return ok


def mapb():
    import oracle as O
    N, K, A, V, Dcap = args.map_pairs, 1024, 32, 2, 4
    a = synth.map_replicas(ctx, N, K, A, V, 0x5EED0004, kmax=256, p_def=0.2)
    b = synth.map_replicas(ctx, N, K, A, V, 0x5EED0004, kmax=256, first_row=N, p_def=0.2)
    Vs = 4

    def offs(x):
        rows = x.def_row.cpu().numpy().astype(np.int64)
        return np.searchsorted(rows, np.arange(N + 1))

    vcl = torch.zeros((N, K, Vs, A), dtype=torch.int64, device=dev)
    vvl = torch.zeros((N, K, Vs), dtype=torch.int64, device=dev)
    vcl[:, :, :V] = a.vclk
    vvl[:, :, :V] = a.vval
    sa = cg.map.MapStates(a.clock, a.ec, vcl, vvl, *slots(offs(a), a.def_clock, a.def_keys, N, 2 * Dcap))
    sb = cg.map.MapStates(b.clock, b.ec, b.vclk, b.vval, *slots(offs(b), b.def_clock, b.def_keys, N, Dcap))
    keep = [x.clone() for x in sa]
    work = cg.map.MapStates(*[x.clone() for x in sa])
    if args.contig:  # self's and other's arrays each in one physically contiguous device block
        def blockify(st):
            pad = lambda n: (n + 511) // 512 * 512  # noqa: E731
            blk = ctx.device_empty((sum(pad(x.numel() * x.element_size() // 8) for x in st),))
            if blk is None:
                return st
            out, at = [], 0
            for x in st:
                n = x.numel() * x.element_size() // 8
                v = blk[at:at + n].view(x.dtype).view(x.shape) if x.element_size() != 8 else blk[at:at + n].view(x.shape)
                v.copy_(x)
                out.append(v)
                at += pad(n)
            return cg.map.MapStates(*out)
        work, sb = blockify(work), blockify(sb)

    def reset():
        for d, s in zip(work, keep):
            d.copy_(s)

    ms = timed(lambda: cg.map.merge_batch(work, sb, ctx=ctx), reset, kernel="map_pair_join")
    spread = dict(SPREAD)
    reset()
    status = cg.map.merge_batch(work, sb, ctx=ctx).cpu().numpy()
    ok = bool((status == 0).all())
    rng = np.random.default_rng(2)

    def obj(st, i):
        n = int(st.def_count[i])
        dc, dk = u64(st.def_clock[i]), u64(st.def_keys[i])
        return O.dense_to_map(u64(st.clock[i]), u64(st.ec[i]), u64(st.vclk[i]), u64(st.vval[i]),
                              [(dc[j], O.bitmap_members(dk[j])) for j in range(n)])

    for i in rng.choice(N, size=args.sample, replace=False):
        i = int(i)
        x = O.dense_to_map(u64(keep[0][i]), u64(keep[1][i]), u64(keep[2][i]), u64(keep[3][i]),
                           [(u64(keep[4][i])[j], O.bitmap_members(u64(keep[5][i])[j])) for j in range(int(keep[6][i]))])
        x.merge(obj(sb, i))
        ok = ok and obj(work, i) == x
    per = K * (A + V * A + V) * 8
    alg = N * (per + K * (A + Vs * A + Vs) * 8 * 2)  # read other, read + write self (Vs slots)
    print(json.dumps({"op": "map_merge_batch", "pairs": N, "keys": K, "actors": A, "kernel_ms_incl_deferred": ms,
                      "algorithmic_bytes": alg, "GBs": alg / ms / 1e6, "frac_of_8TBs": alg / ms / 8e9,
                      "frac_min_max": [alg / spread["ms_max"] / 8e9, alg / spread["ms_min"] / 8e9],
                      "key_pass_ms": spread.get("map_pair_join_ms"), "steps": args.steps,
                      "pair_merges_per_s": N / ms * 1e3, "parity": "ok" if ok else "MISMATCH",
                      "parity_pairs": args.sample}), flush=True)
    return ok


def calib():
    """The same 2-read-1-write byte stream through the plain lattice merge_batch (VClock rows of
    256 actors, crdt_vclock_merge_batch): the practical ceiling of a read-self / read-other /
    write-self pass on this part, beside the 8 TB/s peak."""
    rows = args.orswot_pairs * 4096 * 64 // 256
    a = torch.empty((rows, 256), dtype=torch.int64, device=dev)
    b = torch.empty_like(a)
    cg.synth_fill(ctx, a, 0x5EED0031, 0)
    cg.synth_fill(ctx, b, 0x5EED0032, 0)
    ms = timed(lambda: cg.vclock.merge_batch(a, b, ctx=ctx), lambda: None)
    alg = 3 * a.numel() * 8
    print(json.dumps({"op": "calibration_vclock_merge_batch", "rows": rows, "actors": 256, "ms": ms,
                      "algorithmic_bytes": alg, "GBs": alg / ms / 1e6, "frac_of_8TBs": alg / ms / 8e9}), flush=True)
    del a, b
    torch.cuda.empty_cache()


only = set(args.only.split(","))
good = True
if "calib" in only:
    calib()
if "orswot" in only:
    good = orswot() and good
    torch.cuda.empty_cache()
if "map" in only:
    good = mapb() and good
sys.exit(0 if good else 3)
