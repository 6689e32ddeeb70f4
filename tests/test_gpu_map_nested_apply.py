"""GPU: CmRDT::apply and Causal::forget of Map<K, Map<K2, MVReg<u64>>> (round 5;
crdt_map_nested_apply_batch, crdt_map_nested_forget_batch) — the nested type of the reference's own
Map tests (TMap, /root/reference/test/map.rs:10).

  * The reference's TMap tests as transcribed in tests/test_oracle_map_kat.py (test/map.rs:49-516,
    src/map.rs:381-434, and the quickcheck properties of test/map.rs:524-827 over seeded inputs)
    replayed with EVERY apply, merge and forget of a nested Map running on the GPU: Map.apply /
    Map.merge / Map.forget of the nested instances are routed to the kernels (apply and forget
    through the kernels above, merge through crdt_map_nested_lub_many), so the reference's own
    assertions check them;
  * op streams over many op-replay states in one launch — inner Puts (fresh / seen dots, empty and
    concurrent clocks), inner removes from the future (deferred in the inner Map, re-applied by later
    inner Ups), outer removes (deferred, re-applied by later outer Ups), equal rm clocks — against the
    oracle's Map.apply (map.rs:119-137, :311-348, mvreg.rs:130-166), registers compared in Vec order;
  * whole-state forget against the oracle's Map.forget (map.rs:85-114, mvreg.rs:88-104)."""
import numpy as np
import pytest
import torch

import oracle as O
import test_oracle_map_kat as KAT
from gpu_util import to_dev, to_host
from oracle import Dot, Map, MapRm, MapUp, MVRegPut, VClock
from test_gpu_map_nested import (_slot_deferred, canon, decode_states, gpu_apply, gpu_fold, gpu_forget,
                                 nested_states)

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _nested(m):
    return isinstance(m, Map) and isinstance(m.vnew(), Map)


def _mvmap(m):
    return isinstance(m, Map) and isinstance(m.vnew(), O.MVReg)


# ---- Map<K, MVReg> (config 4's type) through crdt_map_apply_batch / crdt_map_merge_batch -----------
def _mv_ids(maps, ops):
    acts, keys = set(), set()
    for m in maps:
        cl = [m.clock] + list(m.deferred) + [e.clock for e in m.entries.values()]
        cl += [c for e in m.entries.values() for c, _ in e.val.vals]
        for c in cl:
            acts |= set(c.dots)
        keys |= set(m.entries) | {k for ks in m.deferred.values() for k in ks}
    for op in ops:
        if isinstance(op, MapRm):
            acts |= set(op.clock.dots)
            keys |= set(op.keyset)
        else:
            acts |= {op.dot.actor} | set(op.op.clock.dots)
            keys.add(op.key)
    fa = {x: i for i, x in enumerate(sorted(acts or {0}))}
    fk = {x: i for i, x in enumerate(sorted(keys or {0}))}
    return fa, fk


def _mv_conv(m, fa, fk):
    vcm = lambda c: VClock({fa[a]: n for a, n in c.dots.items()})  # noqa: E731
    n = Map(O.MVReg)
    n.clock = vcm(m.clock)
    for rm, ks in m.deferred.items():
        n.deferred[vcm(rm)] = {fk[k] for k in ks}
    for k, e in m.entries.items():
        n.entries[fk[k]] = O.MapEntry(vcm(e.clock), O.MVReg([(vcm(c), v) for c, v in e.val.vals]))
    return n


def _mv_inv(d):
    return {i: x for x, i in d.items()}


def mv_apply(ctx, m, op):
    from test_gpu_map_apply import op_tuple
    from test_gpu_merge_batch import map_egress, map_side
    fa, fk = _mv_ids([m], [op])
    if isinstance(op, MapRm):
        dop = MapRm(VClock({fa[a]: n for a, n in op.clock.dots.items()}), {fk[k] for k in op.keyset})
    else:
        dop = MapUp(Dot(fa[op.dot.actor], op.dot.counter), fk[op.key],
                    MVRegPut(VClock({fa[a]: n for a, n in op.op.clock.dots.items()}), op.op.val))
    st = map_side([_mv_conv(m, fa, fk)], len(fk), len(fa), 8, 16)
    ops = cg.map.encode_ops([[op_tuple(dop)]], len(fa), "cuda:0")
    status = cg.map.apply_batch(st.clock, st.ec, st.vclk, st.vval, st.def_clock, st.def_keys, st.def_count, ops,
                                ctx=ctx).cpu().numpy()
    assert status[0] == 0, status
    return _mv_conv(map_egress(st, 1)[0][0], _mv_inv(fa), _mv_inv(fk))


def mv_merge(ctx, a, b):
    from test_gpu_merge_batch import map_egress, map_side
    fa, fk = _mv_ids([a, b], [])
    me = map_side([_mv_conv(a, fa, fk)], len(fk), len(fa), 8, 16)
    other = map_side([_mv_conv(b, fa, fk)], len(fk), len(fa), 8, 16)
    status = cg.map.merge_batch(me, other, ctx=ctx).cpu().numpy()
    assert status[0] == 0, status
    return _mv_conv(map_egress(me, 1)[0][0], _mv_inv(fa), _mv_inv(fk))


@pytest.fixture
def on_gpu(gpu_ctx, monkeypatch):
    """Route Map.apply / merge / forget of nested Maps (and apply / merge of Map<K, MVReg>: the MVReg Map
    kernels) to the kernels for the duration of a test."""
    orig = {nm: getattr(Map, nm) for nm in ("apply", "merge", "forget")}
    calls = dict.fromkeys(orig, 0)

    def take(self, g):
        self.clock, self.entries, self.deferred = g.clock, g.entries, g.deferred

    def apply(self, op):
        if _mvmap(self):
            calls["apply"] += 1
            return take(self, mv_apply(gpu_ctx, self, op))
        if not _nested(self):
            return orig["apply"](self, op)
        calls["apply"] += 1
        take(self, gpu_apply(gpu_ctx, self, [op]))

    def merge(self, other):
        if _mvmap(self):
            calls["merge"] += 1
            return take(self, mv_merge(gpu_ctx, self, other))
        if not _nested(self):
            return orig["merge"](self, other)
        calls["merge"] += 1
        take(self, gpu_fold(gpu_ctx, [self, other]))

    def forget(self, clock):
        if not _nested(self):
            return orig["forget"](self, clock)
        calls["forget"] += 1
        take(self, gpu_forget(gpu_ctx, self, clock))

    for nm, f in (("apply", apply), ("merge", merge), ("forget", forget)):
        monkeypatch.setattr(Map, nm, f)
    return calls


KATS = ["test_op_exchange_converges_quickcheck1", "test_update", "test_remove", "test_reset_remove_semantics",
        "test_updating_with_current_clock_should_be_a_nop", "test_concurrent_update_and_remove_add_bias",
        "test_op_exchange_commutes_quickcheck1", "test_op_deferred_remove", "test_merge_deferred_remove",
        "test_commute_quickcheck_bug", "test_idempotent_quickcheck_bug1", "test_idempotent_quickcheck_bug2",
        "test_op_exchange_same_as_merge_quickcheck1", "test_idempotent_quickcheck1", "test_is_empty"]


@pytest.mark.parametrize("name", KATS)
def test_reference_map_kats_on_gpu(on_gpu, name):
    getattr(KAT, name)()
    assert on_gpu["apply"] > 0  # the kernels ran


@pytest.mark.parametrize("seed", range(16))
def test_prop_map_merge_laws_all_on_gpu(on_gpu, seed):
    KAT.test_prop_map_merge_laws(seed)
    assert on_gpu["apply"] > 0 and on_gpu["merge"] > 0


@pytest.mark.parametrize("seed", range(12))
def test_prop_map_forget_all_on_gpu(on_gpu, seed):
    KAT.test_prop_map_forget(seed)
    assert on_gpu["forget"] > 0 and on_gpu["merge"] > 0


# ---- op streams over many states in one launch ------------------------------------------------------
def _streams(rng, maps, K, K2, A, T):
    streams, oops = [], []
    for m in maps:
        clk = {a: m.clock.get(a) for a in range(A)}
        icl = {k: {a: e.val.clock.get(a) for a in range(A)} for k, e in m.entries.items()}
        ops, oo = [], []
        for _ in range(T):
            if rng.random() < 0.8:
                a = int(rng.integers(A))
                c = clk[a] + int(rng.integers(1, 3)) if rng.random() < 0.85 else max(clk[a] - int(rng.integers(0, 2)), 1)
                clk[a] = max(clk[a], c)
                k = int(rng.integers(K))
                ic = icl.setdefault(k, {a2: 0 for a2 in range(A)})
                if rng.random() < 0.65:  # inner Up with a Put
                    ia = int(rng.integers(A))
                    icn = ic[ia] + int(rng.integers(1, 3)) if rng.random() < 0.85 else max(ic[ia], 1)
                    ic[ia] = max(ic[ia], icn)
                    j = int(rng.integers(K2))
                    row = {} if rng.random() < 0.1 else {
                        a2: max(0, ic[a2] + int(rng.integers(-2, 2))) for a2 in range(A) if rng.random() < 0.6}
                    row = {a2: v for a2, v in row.items() if v}
                    val = int(rng.integers(100))
                    ops.append(("put", a, c, k, ia, icn, j, row, val))
                    oo.append(MapUp(Dot(a, c), k, MapUp(Dot(ia, icn), j, MVRegPut(VClock(dict(row)), val))))
                else:  # inner Rm, its clock up to 2 ahead of the inner clock seen
                    row = {a2: max(0, ic[a2] + int(rng.integers(-2, 3))) for a2 in range(A) if rng.random() < 0.6}
                    row = {a2: v for a2, v in row.items() if v}
                    js = sorted(set(int(z) for z in rng.choice(K2, size=int(rng.integers(1, 3)), replace=False)))
                    ops.append(("irm", a, c, k, row, js))
                    oo.append(MapUp(Dot(a, c), k, MapRm(VClock(dict(row)), js)))
            else:  # outer Rm
                row = {a2: max(0, clk[a2] + int(rng.integers(-3, 3))) for a2 in range(A) if rng.random() < 0.5}
                row = {a2: v for a2, v in row.items() if v}
                ks = sorted(set(int(z) for z in rng.choice(K, size=int(rng.integers(1, 3)), replace=False)))
                ops.append(("rm", row, ks))
                oo.append(MapRm(VClock(dict(row)), ks))
        streams.append(ops)
        oops.append(oo)
    return streams, oops


def _regs_in_order(m):
    return {(k, j): [(tuple(sorted(c.dots.items())), v) for c, v in ie.val.vals]
            for k, e in m.entries.items() for j, ie in e.val.entries.items()}


def _fits(m):
    return (len(m.deferred) <= 16 and all(len(e.val.deferred) <= 16 for e in m.entries.values())
            and all(len(ie.val.vals) <= 8 for e in m.entries.values() for ie in e.val.entries.values()))


@pytest.mark.parametrize("K,K2,A,seed", [(4, 6, 5, 1), (3, 64, 4, 2), (5, 5, 70, 3),
                                         (3, 200, 5, 4), (2, 256, 130, 5)])  # (K2 > 64: K2w mask words)
def test_map_nested_apply_streams(gpu_ctx, K, K2, A, seed):
    N, T = 24, 30
    maps = [m for m in O.nested_map_objects(N + 8, K, K2, A, seed=80 + seed, steps=200, p_irm=0.5, p_ooo=0.8,
                                            p_rm=0.3) if _fits(m)][:N]
    N = len(maps)
    rng = np.random.default_rng(seed)
    streams, oops = _streams(rng, maps, K, K2, A, T)
    exps = [m.copy() for m in maps]
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    keep = [n for n in range(N) if _fits(exps[n])]
    maps, exps = [maps[n] for n in keep], [exps[n] for n in keep]
    streams = [streams[n] for n in keep]
    st, slots, _ = nested_states(maps, K, K2, A)
    ops = cg.map.encode_nested_ops(streams, A, "cuda:0", K2=K2)
    status = cg.map.nested_apply_batch(st, *slots, ops, ctx=gpu_ctx).cpu().numpy()
    inner_def = outer_def = 0
    for n, exp in enumerate(exps):
        assert status[n] == 0, (n, status[n])
        got = decode_states(st, n, _slot_deferred(slots, n))
        assert canon(got) == canon(exp), n
        assert _regs_in_order(got) == _regs_in_order(exp), n
        inner_def += sum(len(e.val.deferred) for e in exp.entries.values())
        outer_def += len(exp.deferred)
    assert len(exps) >= 12 and inner_def > 0 and outer_def > 0


@pytest.mark.parametrize("mode,K2", [("below", 6), ("all", 6), ("zero", 6), ("zero", 200), ("below", 256)])
def test_map_nested_forget_batch(gpu_ctx, mode, K2):
    K, A = 4, 5
    maps = [m for m in O.nested_map_objects(32, K, K2, A, seed=90, steps=220, p_irm=0.5, p_ooo=0.8, p_rm=0.3)
            if _fits(m)]
    N = len(maps)
    st, _, d = nested_states(maps, K, K2, A)
    rng = np.random.default_rng(len(mode))
    c = d["clock"].astype(np.int64)
    y = {"below": (rng.integers(0, c + 1) * (rng.random(c.shape) < 0.7)).astype(np.uint64),
         "all": d["clock"].copy(), "zero": np.zeros_like(d["clock"])}[mode]
    D = d["def_row"].shape[0]
    dcl = to_dev(d["def_clock"]) if D else None
    dst = torch.from_numpy(d["def_row"].astype(np.int32)).cuda() if D else None
    keep = cg.map.nested_forget_batch(st, to_dev(y), def_clock=dcl, def_state=dst, ctx=gpu_ctx)
    kp = keep.cpu().numpy() if keep is not None else np.zeros(0, np.uint8)
    hc = to_host(dcl) if D else np.zeros((0, A), np.uint64)
    inner_def = 0
    for n, m in enumerate(maps):
        exp = m.copy()
        exp.forget(VClock({a: int(x) for a, x in enumerate(y[n]) if x}))
        dfr = [(hc[j], O.bitmap_members(d["def_keys"][j])) for j in np.flatnonzero(d["def_row"] == n) if kp[j]]
        got = decode_states(st, n, dfr)
        assert canon(got) == canon(exp), n
        assert _regs_in_order(got) == _regs_in_order(exp), n
        inner_def += sum(len(e.val.deferred) for e in exp.entries.values())
    if mode == "zero":
        assert inner_def > 0 and D > 0


def test_map_nested_apply_wide_keyset_malformed(gpu_ctx):
    """K2 = 100 (two mask words per key set): an inner Rm naming key 120 (word 1, past K2) is malformed
    and skipped whole (bit 1); one over keys 3 and 90 (both words) removes both."""
    K, K2, A = 2, 100, 3
    m = Map(lambda: Map(O.MVReg))
    for a, j in ((0, 3), (1, 90), (2, 50)):
        m.apply(MapUp(Dot(a, 1), 0, MapUp(Dot(a, 1), j, MVRegPut(VClock({}), 10 + a))))
    st, slots, _ = nested_states([m, m.copy()], K, K2, A)
    rm_row = {0: 1, 1: 1}
    streams = [[("irm", 0, 2, 0, rm_row, [3, 120])], [("irm", 0, 2, 0, rm_row, [3, 90])]]
    ops = cg.map.encode_nested_ops(streams, A, "cuda:0", K2=K2)
    assert tuple(ops.ikeys.shape) == (2, 2)
    status = cg.map.nested_apply_batch(st, *slots, ops, ctx=gpu_ctx).cpu().numpy()
    assert status[0] & 2 and not status[1] & 2, status
    assert canon(decode_states(st, 0, _slot_deferred(slots, 0))) == canon(m)
    exp = m.copy()
    exp.apply(MapUp(Dot(0, 2), 0, MapRm(VClock(dict(rm_row)), [3, 90])))
    got = decode_states(st, 1, _slot_deferred(slots, 1))
    assert canon(got) == canon(exp)
    assert sorted(got.entries[0].val.entries) == [50]


def test_map_nested_apply_malformed_and_capacity(gpu_ctx):
    """Malformed ops are skipped whole (bit 1); an outer deferred list past Dcap is flagged (bit 0);
    a register past 8 values is flagged (bit 4) with the value not added."""
    K, K2, A = 2, 3, 4
    m = Map(lambda: Map(O.MVReg))
    st, slots, _ = nested_states([m, m.copy(), m.copy()], K, K2, A)
    # nine pairwise-concurrent Put clocks on one register: the ninth value does not fit
    concurrent = [("put", 0, i + 1, 0, i % A, i + 1, 0, {0: i + 1, 1: 9 - i}, i) for i in range(9)]
    streams = [
        [("put", 9, 1, 0, 0, 1, 0, {0: 1}, 5), ("put", 0, 1, 7, 0, 1, 0, {0: 1}, 5),
         ("put", 0, 1, 0, 0, 1, 9, {0: 1}, 5), ("irm", 0, 1, 0, {0: 1}, [5]), ("put", 1, 1, 1, 2, 3, 2, {2: 3}, 7)],
        [("rm", {0: 5 + i}, [i % K]) for i in range(18)],
        concurrent,
    ]
    ops = cg.map.encode_nested_ops(streams, A, "cuda:0")
    status = cg.map.nested_apply_batch(st, *slots, ops, ctx=gpu_ctx).cpu().numpy()
    assert status[0] == 2 and status[1] == 1, status
    got = decode_states(st, 0, _slot_deferred(slots, 0))
    assert set(got.entries) == {1} and got.entries[1].val.entries[2].val.vals[0][1] == 7
    assert int(slots[2][1]) == 16
    assert status[2] == 16, status
    got = decode_states(st, 2, _slot_deferred(slots, 2))
    assert [v for _, v in got.entries[0].val.entries[0].val.vals] == list(range(8))


def test_map_nested_apply_unapplied_input_deferred(gpu_ctx):
    """Outer removes in the input never applied to their keys: the first Up's full apply_deferred pass
    applies them (the later passes re-forget the Up's key only)."""
    K, K2, A, T = 4, 6, 5, 20
    maps = [m for m in O.nested_map_objects(24, K, K2, A, seed=84, steps=200, p_irm=0.5, p_ooo=0.8, p_rm=0.3)
            if _fits(m) and len(m.deferred) < 16][:16]
    rng = np.random.default_rng(85)
    for m in maps:
        row = {0: m.clock.get(0) + 1, 1: m.clock.get(1) + 1}
        m.deferred[VClock(row)] = set(int(k) for k in rng.choice(K, size=2, replace=False))
    streams, oops = _streams(rng, maps, K, K2, A, T)
    exps = [m.copy() for m in maps]
    for n, e in enumerate(exps):
        for op in oops[n]:
            e.apply(op)
    keep = [n for n, e in enumerate(exps) if _fits(e)]
    st, slots, _ = nested_states([maps[n] for n in keep], K, K2, A)
    ops = cg.map.encode_nested_ops([streams[n] for n in keep], A, "cuda:0")
    status = cg.map.nested_apply_batch(st, *slots, ops, ctx=gpu_ctx).cpu().numpy()
    for i, n in enumerate(keep):
        assert status[i] == 0, (i, status[i])
        got = decode_states(st, i, _slot_deferred(slots, i))
        assert canon(got) == canon(exps[n]) and _regs_in_order(got) == _regs_in_order(exps[n]), n
    assert len(keep) >= 8


def test_map_nested_apply_long_outer_deferred_list(gpu_ctx):
    """More outer deferred removes than the 16 slots the kernel holds in LDS (round 6: the rest of Dcap
    used in place in the caller's slot arrays): outer Rms from the far future on actor 0 (Ups on actors
    1..), 20+ removes per state at Dcap = 48, equal to the oracle's Map.apply."""
    K, K2, A, T, Dcap = 4, 5, 4, 60, 48
    maps = [m for m in O.nested_map_objects(14, K, K2, A, seed=85, steps=150, p_irm=0.4, p_ooo=0.5, p_rm=0.2)
            if _fits(m)][:10]
    N = len(maps)
    rng = np.random.default_rng(19)
    streams, oops = [], []
    for m in maps:
        clk = {a: m.clock.get(a) for a in range(A)}
        ops, oo = [], []
        for i in range(T):
            if rng.random() < 0.55:
                row = {0: clk[0] + 1000 + i}
                ks = sorted(set(int(z) for z in rng.choice(K, size=int(rng.integers(1, 3)), replace=False)))
                ops.append(("rm", row, ks))
                oo.append(MapRm(VClock(dict(row)), ks))
            else:
                a = int(rng.integers(1, A))
                c = clk[a] + 1
                clk[a] = c
                k, j, ia = int(rng.integers(K)), int(rng.integers(K2)), int(rng.integers(1, A))
                icn, val = 500 + i, int(rng.integers(100))
                ops.append(("put", a, c, k, ia, icn, j, {}, val))
                oo.append(MapUp(Dot(a, c), k, MapUp(Dot(ia, icn), j, MVRegPut(VClock({}), val))))
        streams.append(ops)
        oops.append(oo)
    exps = [m.copy() for m in maps]
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    st, slots, _ = nested_states(maps, K, K2, A, Dcap=Dcap)
    ops = cg.map.encode_nested_ops(streams, A, "cuda:0")
    status = cg.map.nested_apply_batch(st, *slots, ops, ctx=gpu_ctx).cpu().numpy()
    longest = 0
    for n, exp in enumerate(exps):
        assert status[n] == 0, (n, status[n])
        got = decode_states(st, n, _slot_deferred(slots, n))
        assert canon(got) == canon(exp), n
        longest = max(longest, len(exp.deferred))
    assert N >= 8 and 20 <= longest <= Dcap
