"""CmRDT::apply, Causal::forget and the serde wire form of the value-typed Maps on one MI355X (round 5):
  * crdt_map_counter_apply_batch — Map<K, PNCounter>, N states x T ops (85% Ups with a fresh Map dot
    and a counter dot in either direction, 5% of them seen, 15% Map Rms, some from the future);
  * crdt_map_orswot_apply_batch — Map<K, Orswot<M>>: Orswot Adds, Orswot Rms, Map Rms;
  * crdt_map_nested_apply_batch — Map<K, Map<K2, MVReg>> (the reference's TMap): inner Puts, inner
    Rms, outer Rms; then crdt_map_nested_forget_batch of the results;
  * crdt_map_{counter,nested}_egress / _ingest of the applied states (round trip checked equal).
States start empty and are reset before every rep; streams are generated on the host (numpy) with
the same shape as the oracle tests'.  HIP-event kernel time (ctx timing); parity of a state sample
against the oracle's Map.apply / forget (reference-shaped objects).  One JSON line per op."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-crdt_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import crdts_gpu as cg  # noqa: E402
from crdts_gpu import wire  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--states", type=int, default=65536)
ap.add_argument("--ops", type=int, default=64)
ap.add_argument("--nested-states", type=int, default=32768)
ap.add_argument("--nested-ops", type=int, default=32)
ap.add_argument("--actors", type=int, default=32)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--sample", type=int, default=48)
ap.add_argument("--dcap", type=int, default=64,
                help="deferred slots per state (the kernels hold 16 in LDS and use the rest in place)")
args = ap.parse_args()
A = args.actors
torch.cuda.set_device(0)
ctx = cg.Context(0)
rng = np.random.default_rng(0x5EED00A1)
dev = "cuda"
i64 = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
i32 = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.int32)).to(dev)  # noqa: E731
u8 = lambda x: torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint8)).to(dev)  # noqa: E731


def timed(name, reset, run):
    reset()
    run()
    torch.cuda.synchronize()
    ctx.timing_reset()
    out = None
    for _ in range(args.reps):
        reset()
        torch.cuda.synchronize()
        ctx.set_timing(True)
        out = run()
        torch.cuda.synchronize()
        ctx.set_timing(False)
    ms, n = ctx.timing(name)
    return ms / n, out


def rm_rows(n, t_of_op, ahead=3):
    """n rm clock rows: each actor present w.p. 0.3 with a counter up to the op's index + `ahead`."""
    rows = rng.integers(1, np.maximum(t_of_op + ahead, 2)[:, None], size=(n, A)).astype(np.uint64)
    rows[rng.random((n, A)) > 0.3] = 0
    return rows


def common(N, T, p_rm):
    n = N * T
    kind = (rng.random(n) < p_rm).astype(np.uint8)
    t = np.tile(np.arange(T), N)
    actor = rng.integers(0, A, n)
    counter = (t + 1).astype(np.uint64)
    counter[rng.random(n) < 0.05] = 1  # seen dots
    return n, kind, t, actor, counter


def emit(name, N, T, ms, status, ok, extra):
    st = status.cpu().numpy()
    print(json.dumps(dict({"op": name, "states": N, "ops_per_state": T, "actors": A, "kernel_us": ms * 1e3,
                           "ops_per_s": N * T / (ms / 1e3), "status_nonzero_states": int((st != 0).sum()),
                           "parity": "ok" if ok else "MISMATCH"}, **extra)), flush=True)


import oracle as O  # noqa: E402  (the checker only)

# ---- Map<K, PNCounter> -------------------------------------------------------------------------------
N, T, K, W = args.states, args.ops, 64, 2
n, kind, t, actor, counter = common(N, T, 0.15)
rm = np.flatnonzero(kind == 1)
pool = rm_rows(len(rm), t[rm], ahead=1)
clk_row = np.zeros(n, np.int64)
clk_row[rm] = np.arange(len(rm))
key = rng.integers(0, K, n)
key_off = np.concatenate([[0], np.cumsum(kind)]).astype(np.uint64)
ops = cg.map.MapCounterOpBatch(i64(np.arange(N + 1) * T), u8(kind), i32(actor), i64(counter), i32(key),
                               i32(rng.integers(0, A, n)), i64(rng.integers(1, 1 << 20, n)), u8(rng.integers(0, 2, n)),
                               i32(clk_row), i64(pool if len(pool) else np.zeros((1, A))), i64(key_off), i32(key[rm]))
z = lambda *s: torch.zeros(s, dtype=torch.int64, device=dev)  # noqa: E731
Dcap = args.dcap
cs = [z(N, A), z(N, K, A), z(N, K, W, A), z(N, Dcap, A), z(N, Dcap, 1), torch.zeros(N, dtype=torch.int32, device=dev)]
ms, status = timed("map_counter_apply", lambda: [x.zero_() for x in cs],
                   lambda: cg.map.counter_apply_batch(*cs, ops, ctx=ctx))
h = {f: getattr(ops, f).cpu().numpy() for f in ops._fields}
sample = rng.choice(N, size=args.sample, replace=False)
ok = True
hc, he, hv = (x.cpu().numpy().view(np.uint64) for x in cs[:3])
hdc, hdk, hcnt = cs[3].cpu().numpy().view(np.uint64), cs[4].cpu().numpy().view(np.uint64), cs[5].cpu().numpy()
st_np = status.cpu().numpy()
bad = []
for s in sample:
    if st_np[s]:  # (a state with a nonzero status is a failure of the parity check)
        bad.append(int(s))
        continue
    m = O.Map(O.PNCounter)
    for o in range(s * T, (s + 1) * T):
        if h["kind"][o] == 0:
            d = O.PNCounter.POS if h["vdir"][o] == 0 else O.PNCounter.NEG
            m.apply(O.MapUp(O.Dot(int(h["actor"][o]), int(h["counter"][o].view(np.uint64))), int(h["key"][o]),
                            (O.Dot(int(h["vactor"][o]), int(h["vcounter"][o])), d)))
        else:
            row = h["clk_pool"][h["clk_row"][o]].view(np.uint64)
            m.apply(O.MapRm(O.VClock({a: int(v) for a, v in enumerate(row) if v}), {int(h["keys"][h["key_off"][o]])}))
    dfr = [(hdc[s, i], O.bitmap_members(hdk[s, i])) for i in range(int(hcnt[s]))]
    if O.dense_to_map_counter(hc[s], he[s], hv[s], dfr) != m:
        bad.append(int(s))
ok = not bad
emit("map_counter_apply_batch (PNCounter values)", N, T, ms, status, ok, {"keys": K, "dcap": Dcap,
     "deferred_left": int(hcnt.sum()), "deferred_max": int(hcnt.max()), "parity_states": len(sample),
     "mismatched": bad})
# the wire round trip of those states
st_c = wire.MapCounterFrames(*cs)
aids = i32(np.arange(A) * 7 + 3)
kids = i32(np.arange(K) * 5 + 1)
off, data = wire.map_counter_egress(st_c, aids, kids, ctx=ctx)
ms_e, _ = timed("wire_egress", lambda: None, lambda: wire.map_counter_egress(st_c, aids, kids, ctx=ctx))
ms_i, (back, bst) = timed("wire_ingest", lambda: None,
                          lambda: wire.map_counter_ingest(data, off, aids, kids, W, Dcap, ctx=ctx))
same = all(bool(torch.equal(a_, b_)) for a_, b_ in zip(back, st_c)) and not bool((bst != 0).any())
print(json.dumps({"op": "map_counter_egress / _ingest (PNCounter values)", "states": N, "frame_bytes": int(data.numel()),
                  "egress_us": ms_e * 1e3, "ingest_us": ms_i * 1e3, "egress_GBs_of_frames": data.numel() / ms_e / 1e6,
                  "ingest_GBs_of_frames": data.numel() / ms_i / 1e6,
                  "round_trip": "ok" if same else "MISMATCH"}), flush=True)
del cs, st_c, back, data, ops

# ---- Map<K, Orswot<M>> -----------------------------------------------------------------------------
N, T, K, M = args.states, args.ops, 16, 8
n, kind, t, actor, counter = common(N, T, 0.15)
vkind = ((rng.random(n) < 0.2) & (kind == 0)).astype(np.uint8)
need = np.flatnonzero((kind == 1) | (vkind == 1))
pool = rm_rows(len(need), t[need], ahead=1)
clk_row = np.zeros(n, np.int64)
clk_row[need] = np.arange(len(need))
key = rng.integers(0, K, n)
rmk = np.flatnonzero(kind == 1)
key_off = np.concatenate([[0], np.cumsum(kind)]).astype(np.uint64)
mem = rng.integers(0, M, n)
has_mem = (kind == 0).astype(np.uint64)
mem_off = np.concatenate([[0], np.cumsum(has_mem)]).astype(np.uint64)
vcounter = (t + 1).astype(np.uint64)
ops = cg.map.MapOrswotOpBatch(i64(np.arange(N + 1) * T), u8(kind), i32(actor), i64(counter), i32(key), u8(vkind),
                              i32(rng.integers(0, A, n)), i64(vcounter), i32(clk_row), i64(pool), i64(key_off),
                              i32(key[rmk]), i64(mem_off), i32(mem[kind == 0]))
Mw = 1
os_ = [z(N, A), z(N, K, A), z(N, K, A), z(N, K, M, A), torch.zeros((N, K), dtype=torch.int32, device=dev),
       z(N, K, 16, A), z(N, K, 16)]
sl = [z(N, Dcap, A), z(N, Dcap, 1), torch.zeros(N, dtype=torch.int32, device=dev)]
res = cg.map.MapOrswotLub(*os_, None, None, None)
ms, status = timed("map_orswot_apply", lambda: [x.zero_() for x in os_ + sl],
                   lambda: cg.map.orswot_apply_batch(res, *sl, ops, ctx=ctx))
h = {f: getattr(ops, f).cpu().numpy() for f in ops._fields}
hs = [x.cpu().numpy() for x in os_]
hs = [x.view(np.uint64) if x.dtype == np.int64 else x for x in hs]
hdc, hdk, hcnt = sl[0].cpu().numpy().view(np.uint64), sl[1].cpu().numpy().view(np.uint64), sl[2].cpu().numpy()
ok = True
st_np = status.cpu().numpy()
for s in sample:
    if st_np[s]:  # (a state with a nonzero status is a failure of the parity check)
        ok = False
        continue
    m = O.Map(O.Orswot)
    for o in range(s * T, (s + 1) * T):
        row = h["clk_pool"][h["clk_row"][o]].view(np.uint64)
        rc = O.VClock({a: int(v) for a, v in enumerate(row) if v})
        if h["kind"][o] == 1:
            m.apply(O.MapRm(rc, {int(h["keys"][h["key_off"][o]])}))
            continue
        ms_ = {int(h["mems"][h["mem_off"][o]])}
        vop = (O.OrswotAdd(O.Dot(int(h["vactor"][o]), int(h["vcounter"][o])), ms_) if h["vkind"][o] == 0
               else O.OrswotRm(rc, ms_))
        m.apply(O.MapUp(O.Dot(int(h["actor"][o]), int(h["counter"][o])), int(h["key"][o]), vop))
    vd = {k: [(hs[5][s, k, i], O.bitmap_members(hs[6][s, k, i:i + 1])) for i in range(int(hs[4][s, k]))]
          for k in range(K)}
    dfr = [(hdc[s, i], O.bitmap_members(hdk[s, i])) for i in range(int(hcnt[s]))]
    g = O.dense_to_map_orswot(hs[0][s], hs[1][s], hs[2][s], hs[3][s], vd, dfr)
    ok &= g.clock == m.clock and g.entries == m.entries and g.deferred == m.deferred
emit("map_orswot_apply_batch", N, T, ms, status, ok, {"keys": K, "members": M, "dcap": Dcap})
del os_, sl, res, ops

# ---- Map<K, Map<K2, MVReg>> ---------------------------------------------------------------------------
N, T, K, K2 = args.nested_states, args.nested_ops, 16, 8
n, kind, t, actor, counter = common(N, T, 0.15)
ikind = ((rng.random(n) < 0.2) & (kind == 0)).astype(np.uint8)
iactor = rng.integers(0, A, n)
icounter = (t + 1).astype(np.uint64)
pool = rm_rows(n, t, ahead=2)
put = (kind == 0) & (ikind == 0)
pool[put] = 0
pool[np.flatnonzero(put), iactor[put]] = icounter[put]  # a Put's clock: its own dot (a fresh write)
key = rng.integers(0, K, n)
rmk = np.flatnonzero(kind == 1)
key_off = np.concatenate([[0], np.cumsum(kind)]).astype(np.uint64)
ikeys = (np.uint64(1) << rng.integers(0, K2, n).astype(np.uint64)) * (ikind == 1)
ops = cg.map.MapNestedOpBatch(i64(np.arange(N + 1) * T), u8(kind), i32(actor), i64(counter), i32(key), u8(ikind),
                              i32(iactor), i64(icounter), i32(rng.integers(0, K2, n)), i64(rng.integers(0, 1000, n)),
                              i64(ikeys), i32(np.arange(n)), i64(pool), i64(key_off), i32(key[rmk]))
ns = [z(N, A), z(N, K, A), z(N, K, A), z(N, K, K2, A), z(N, K, K2, 8, A), z(N, K, K2, 8),
      torch.zeros((N, K, K2), dtype=torch.int32, device=dev), torch.zeros((N, K), dtype=torch.int32, device=dev),
      z(N, K, 16, A), z(N, K, 16)]
sl = [z(N, Dcap, A), z(N, Dcap, 1), torch.zeros(N, dtype=torch.int32, device=dev)]
st_n = wire.MapNestedFrames(*ns, *sl)
ms, status = timed("map_nested_apply", lambda: [x.zero_() for x in ns + sl],
                   lambda: cg.map.nested_apply_batch(st_n, *sl, ops, ctx=ctx))
h = {f: getattr(ops, f).cpu().numpy() for f in ops._fields}
snap = [x.clone() for x in ns + sl]


def host_state(tensors, s):
    from test_gpu_map_nested import _States, decode_states
    st = _States(*(x[s:s + 1] for x in tensors[:10]))  # (one state to the host, not the batch)
    dc, dk, cnt = (x[s].cpu().numpy() for x in tensors[10:])
    dfr = [(dc[i].view(np.uint64), O.bitmap_members(dk[i].view(np.uint64))) for i in range(int(cnt))]
    return decode_states(st, 0, dfr)


def nested_obj_ops(s):
    out = []
    for o in range(s * T, (s + 1) * T):
        row = h["clk_pool"][h["clk_row"][o]].view(np.uint64)
        rc = O.VClock({a: int(v) for a, v in enumerate(row) if v})
        if h["kind"][o] == 1:
            out.append(O.MapRm(rc, {int(h["keys"][h["key_off"][o]])}))
        elif h["ikind"][o] == 1:
            js = {j for j in range(K2) if (int(h["ikeys"][o].view(np.uint64)) >> j) & 1}
            out.append(O.MapUp(O.Dot(int(h["actor"][o]), int(h["counter"][o])), int(h["key"][o]), O.MapRm(rc, js)))
        else:
            out.append(O.MapUp(O.Dot(int(h["actor"][o]), int(h["counter"][o])), int(h["key"][o]),
                               O.MapUp(O.Dot(int(h["iactor"][o]), int(h["icounter"][o])), int(h["ikey"][o]),
                                       O.MVRegPut(rc, int(h["val"][o])))))
    return out


from test_gpu_map_nested import canon  # noqa: E402

ok = True
st_np = status.cpu().numpy()
exps = {}
for s in sample % N:
    if st_np[s]:  # (a state with a nonzero status is a failure of the parity check)
        ok = False
        continue
    m = O.Map(lambda: O.Map(O.MVReg))
    for op in nested_obj_ops(int(s)):
        m.apply(op)
    exps[int(s)] = m
    ok &= canon(host_state(ns + sl, int(s))) == canon(m)
emit("map_nested_apply_batch", N, T, ms, status, ok, {"keys": K, "inner_keys": K2, "dcap": Dcap})
# the wire round trip, then forget
aids = i32(np.arange(A) * 7 + 3)
kids = i32(np.arange(K) * 5 + 1)
iids = i32(np.arange(K2) * 3 + 2)
off, data = wire.map_nested_egress(st_n, aids, kids, iids, ctx=ctx)
ms_e, _ = timed("wire_egress", lambda: None, lambda: wire.map_nested_egress(st_n, aids, kids, iids, ctx=ctx))
ms_i, (back, bst) = timed("wire_ingest", lambda: None,
                          lambda: wire.map_nested_ingest(data, off, aids, kids, iids, Dcap, ctx=ctx))
same = all(bool(torch.equal(a_, b_)) for a_, b_ in zip(back, st_n)) and not bool((bst != 0).any())
print(json.dumps({"op": "map_nested_egress / _ingest", "states": N, "frame_bytes": int(data.numel()),
                  "egress_us": ms_e * 1e3, "ingest_us": ms_i * 1e3, "egress_GBs_of_frames": data.numel() / ms_e / 1e6,
                  "ingest_GBs_of_frames": data.numel() / ms_i / 1e6,
                  "round_trip": "ok" if same else "MISMATCH"}), flush=True)
y = (ns[0] // 2).contiguous()  # forget half of each state's history
ms, _ = timed("map_nested_forget", lambda: [d.copy_(s_) for d, s_ in zip(ns + sl, snap)],
              lambda: cg.map.nested_forget_batch(st_n, y, ctx=ctx))
hy = y.cpu().numpy().view(np.uint64)
okf = True
for s, m in exps.items():
    m.forget(O.VClock({a: int(v) for a, v in enumerate(hy[s]) if v}))
    g = host_state(ns + sl, s)
    okf &= canon(g)[:2] == canon(m)[:2]  # clock and entries (the outer removes are the pool argument, omitted)
print(json.dumps({"op": "map_nested_forget_batch", "states": N, "kernel_us": ms * 1e3,
                  "states_per_s": N / (ms / 1e3), "parity": "ok" if okf else "MISMATCH",
                  "parity_states": len(exps)}), flush=True)
