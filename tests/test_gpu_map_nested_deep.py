"""GPU: Map<K, Map<K2, MVReg>> with more than 16 inner deferred removes on one key (round 6).

The reference's inner Map keeps any number of deferred removes (map.rs:37, apply_keyset_rm :318-348,
merge :140-220); the nested layouts carry Id inner slots per key (crdt_map_nested_states.Id /
crdt_map_nested_out.Id, 16 by default).  The fold keeps 16 in LDS and re-folds, exactly, the keys whose
inner list passed 16 with all Id; the apply, forget, merge_batch and the wire form use all Id.  Every
case is checked against the oracle's Map (a restatement of map.rs / mvreg.rs)."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host
from oracle import Dot, MapRm, MapUp, MVRegPut, VClock

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import wire  # noqa: E402
from test_gpu_map_nested import _slot_deferred, canon, decode_states, nested_states  # noqa: E402


def _deep_nested(rng, R, K, K2, A, per=8):
    """R replicas (replica r writes as actor r: A >= R) whose keys' inner Maps hold up to `per`
    deferred removes each, clocks from the far future on actor 0 (a fold unions them)."""
    assert A >= R
    maps = []
    for r in range(R):
        m = O.Map(lambda: O.Map(O.MVReg))
        m.clock = VClock({r: 5})
        for k in range(K):
            if rng.random() < 0.9:
                inner = O.Map(O.MVReg)
                inner.clock = VClock({r: int(rng.integers(1, 4))})
                for j in range(K2):
                    if rng.random() < 0.4:
                        c = VClock({r: int(rng.integers(1, 4))})
                        inner.entries[j] = O.MapEntry(c.copy(), O.MVReg([(c, int(rng.integers(100)))]))
                for _ in range(int(rng.integers(1, per + 1))):
                    rm = {0: int(rng.integers(100, 100000))}
                    if rng.random() < 0.5:
                        rm[int(rng.integers(1, A))] = int(rng.integers(1, 3))
                    inner.deferred[VClock(rm)] = set(int(x) for x in rng.choice(K2, size=int(rng.integers(1, min(K2, 3) + 1)),
                                                                             replace=False))
                m.entries[k] = O.MapEntry(VClock({r: int(rng.integers(1, 5))}), inner)
        maps.append(m)
    return maps


def _longest(maps):
    return max([len(e.val.deferred) for x in maps for e in x.entries.values()] + [0])


def _fold(ctx, maps, K, K2, A, G=1, id_cap="auto", check=True, v_cap=8, V=8):
    d = O.nested_map_to_dense(maps, K, K2, A, V)
    R = len(maps) // G
    shp = lambda x: to_dev(x.reshape((G, R) + x.shape[1:]))  # noqa: E731
    Di = int(d["id_off"][-1])
    ikw = dict(id_clock=to_dev(d["id_clock"]), id_keys=to_dev(d["id_keys"])) if Di else {}
    return cg.map.nested_lub_many(shp(d["clock"]), shp(d["ec"]), shp(d["ic"]), shp(d["iec"]), shp(d["ivc"]),
                                  shp(d["ivv"]), to_dev(d["id_off"]), ctx=ctx, check=check, id_cap=id_cap,
                                  v_cap=v_cap, **ikw)


def _decode_fold(res, g):
    sq = res.clock.dim() == 1
    st = res._replace(**{f: getattr(res, f)[None] for f in ("clock", "ec", "ic", "iec", "ivc", "ivv", "nval", "id_n",
                                                              "id_clock", "id_keys")}) if sq else res
    return decode_states(st, g, [])


@pytest.mark.parametrize("R,K,K2,A,seed,id_cap", [(10, 3, 6, 12, 1, "auto"), (12, 2, 5, 12, 2, 96),
                                                  (6, 2, 100, 8, 3, "auto"), (6, 2, 5, 80, 4, "auto")])
def test_map_nested_fold_past_16_inner(gpu_ctx, R, K, K2, A, seed, id_cap):
    """Keys whose inner Map ends with more than 16 deferred removes (A past one lane word, K2 past one
    mask word among the cases): the deep pass's result equals the oracle's left fold."""
    rng = np.random.default_rng(seed)
    maps = _deep_nested(rng, R, K, K2, A)
    exp = O.map_fold_objects(maps)
    assert _longest([exp]) > 16
    res = _fold(gpu_ctx, maps, K, K2, A, id_cap=id_cap)
    assert int(res.flags.cpu().numpy()[0]) == 0
    assert canon(_decode_fold(res, 0)) == canon(exp)


def test_map_nested_fold_mixed_depths_and_default_flag(gpu_ctx):
    """G = 4 groups of mixed depth re-fold only the deep keys; the default 16 slots flag bit 4."""
    K, K2, A, R = 3, 6, 8, 8
    rng = np.random.default_rng(7)
    parts = [_deep_nested(rng, R, K, K2, A, per=8 if g % 2 == 0 else 1) for g in range(4)]
    res = _fold(gpu_ctx, [m for p in parts for m in p], K, K2, A, G=4, id_cap=80)
    for g in range(4):
        assert canon(_decode_fold(res, g)) == canon(O.map_fold_objects(parts[g])), g
    assert _longest([O.map_fold_objects(parts[0])]) > 16 >= _longest([O.map_fold_objects(parts[1])])
    with pytest.raises(RuntimeError, match="id_cap"):
        _fold(gpu_ctx, parts[0], K, K2, A, id_cap=16)


def test_map_nested_apply_past_16_inner(gpu_ctx):
    """Inner Rms from the far future on one key, 40 per state, on states with Id = 64 inner slots; later
    Puts re-apply every one of them; 16-slot states flag the overflow (status bit 0)."""
    N, K, K2, A, T = 8, 3, 6, 8, 60
    rng = np.random.default_rng(13)
    base = [O.map_fold_objects([m]) for m in _deep_nested(rng, N, K, K2, A, per=1)]  # (states a replica holds)
    exps = [m.copy() for m in base]
    streams, oops = [], []
    for x in exps:
        clk = {a: x.clock.get(a) for a in range(A)}
        ops, oo = [], []
        for i in range(T):
            a = int(rng.integers(A))
            clk[a] += 1
            if i % 3 != 2:  # an inner Rm from the future on key 0
                row = {0: 1000 + i, int(rng.integers(1, A)): 1}
                js = sorted(set(int(z) for z in rng.choice(K2, size=int(rng.integers(1, 3)), replace=False)))
                ops.append(("irm", a, clk[a], 0, row, js))
                oo.append(MapUp(Dot(a, clk[a]), 0, MapRm(VClock(row), js)))
            else:  # an inner Put on key 0 (re-applies the inner removes) or another key
                k = 0 if rng.random() < 0.7 else int(rng.integers(1, K))
                ia, j = int(rng.integers(1, A)), int(rng.integers(K2))
                ops.append(("put", a, clk[a], k, ia, 50 + i, j, {}, 7 + i))
                oo.append(MapUp(Dot(a, clk[a]), k, MapUp(Dot(ia, 50 + i), j, MVRegPut(VClock({}), 7 + i))))
        streams.append(ops)
        oops.append(oo)
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    assert 16 < _longest(exps) <= 64
    st, slots, _ = nested_states(base, K, K2, A, Dcap=4, Id=64)
    enc = cg.map.encode_nested_ops(streams, A, "cuda:0", K2=K2)
    status = cg.map.nested_apply_batch(st, *slots, enc, ctx=gpu_ctx).cpu().numpy()
    for n in range(N):
        assert status[n] == 0, (n, status[n])
        assert canon(decode_states(st, n, _slot_deferred(slots, n))) == canon(exps[n]), n
    st16, slots16, _ = nested_states(base, K, K2, A, Dcap=4)
    s16 = cg.map.nested_apply_batch(st16, *slots16, enc, ctx=gpu_ctx).cpu().numpy()
    assert all(x & 1 for x in s16)
    assert int(st16.id_n.max()) <= 16


def test_map_nested_forget_merge_wire_past_16_inner(gpu_ctx):
    """Deep states (Id = 128) through the wire form, merge_batch and forget, each equal to the oracle."""
    K, K2, A, R, N = 3, 6, 9, 9, 4
    rng = np.random.default_rng(21)
    groups = [_deep_nested(rng, R, K, K2, A) for _ in range(2 * N)]
    folds = [O.map_fold_objects(g) for g in groups]
    assert _longest(folds) > 16
    res = _fold(gpu_ctx, [m for g in groups for m in g], K, K2, A, G=2 * N, id_cap=128)
    Kw = (K + 63) // 64
    z = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    slots = lambda: (z(N, 2, A), z(N, 2, Kw), torch.zeros(N, dtype=torch.int32, device="cuda:0"))  # noqa: E731
    me = wire.MapNestedFrames(*[t[:N].contiguous() for t in res[:10]], *slots())
    other = wire.MapNestedFrames(*[t[N:].contiguous() for t in res[:10]], *slots())
    r2 = np.random.default_rng(3)
    ad = torch.tensor(np.sort(r2.choice(2**31, size=A, replace=False)), dtype=torch.int32, device="cuda:0")
    kd = torch.tensor(np.sort(r2.choice(2**31, size=K, replace=False)), dtype=torch.int32, device="cuda:0")
    idd = torch.tensor(np.sort(r2.choice(2**31, size=K2, replace=False)), dtype=torch.int32, device="cuda:0")
    off, data = wire.map_nested_egress(me, ad, kd, idd, ctx=gpu_ctx)
    back, st = wire.map_nested_ingest(data, off, ad, kd, idd, 2, ctx=gpu_ctx, id_cap=128)
    assert (st.cpu().numpy() == 0).all()
    for i in range(N):
        assert canon(decode_states(back, i, [])) == canon(folds[i]), i
    status = cg.map.nested_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    exps = []
    for i in range(N):
        exp = folds[i].copy()
        exp.merge(folds[N + i].copy())
        exps.append(exp)
        assert canon(decode_states(me, i, [])) == canon(exp), i
    assert _longest(exps) > 16
    y = torch.zeros(A, dtype=torch.int64, device="cuda:0")
    y[0] = 50000
    cg.map.nested_forget_batch(me, y, ctx=gpu_ctx)
    for i in range(N):
        exps[i].forget(VClock({0: 50000}))
        assert canon(decode_states(me, i, [])) == canon(exps[i]), i


def test_map_nested_fold_past_256_live_removes(gpu_ctx):
    """320 live outer removes naming one key (flags bit 3 before round 6): the deep pass holds the
    group's whole remove list; equal to the oracle's fold, outer survivors included."""
    from test_gpu_map_orswot_deep import _many_live
    from test_gpu_map_nested import gpu_fold

    def val(r, k):
        inner = O.Map(O.MVReg)
        inner.clock = VClock({r: 2})
        c = VClock({r: 1 + k % 2})
        inner.entries[r] = O.MapEntry(c.copy(), O.MVReg([(c, 7 + r)]))  # (one writer per inner key)
        return inner
    maps = _many_live(40, 3, lambda *a: val(*a) if a else O.Map(O.MVReg))
    exp = O.map_fold_objects(maps)
    assert len(exp.deferred) > 256
    assert canon(gpu_fold(gpu_ctx, maps)) == canon(exp)


def _many_values(R, K2, per=1):
    """R replicas (actor r) each writing `per` concurrent values to inner key 0 of outer key 0 (clocks
    {r: 1 + i} per writer... one writer per value: actor r * per + i), so a fold holds R * per values."""
    maps = []
    for r in range(R):
        m = O.Map(lambda: O.Map(O.MVReg))
        inner = O.Map(O.MVReg)
        acts = [r * per + i for i in range(per)]
        m.clock = VClock({a: 2 for a in acts})
        inner.clock = VClock({a: 1 for a in acts})
        reg = O.MVReg([(VClock({a: 1}), 100 + a) for a in acts])
        inner.entries[0] = O.MapEntry(VClock({a: 1 for a in acts}), reg)
        inner.entries[1 + r % (K2 - 1)] = O.MapEntry(VClock({acts[0]: 1}), O.MVReg([(VClock({acts[0]: 1}), 7)]))
        m.entries[0] = O.MapEntry(VClock({a: 2 for a in acts}), inner)
        maps.append(m)
    return maps


def _max_vals(m):
    return max(len(ie.val.vals) for e in m.entries.values() for ie in e.val.entries.values())


def test_map_nested_fold_past_8_values(gpu_ctx):
    """20 concurrent writers of one register (flags bit 6 before round 6): v_cap = 32 slots, the keys past
    8 values re-folded in the deep pass; inputs with 12 values per register (V = 12 > 8) fold in the deep
    pass alone; equal to the oracle, and the default 8 slots flag the overflow."""
    maps = _many_values(20, 4)
    exp = O.map_fold_objects(maps)
    assert _max_vals(exp) == 20
    res = _fold(gpu_ctx, maps, 1, 4, 20, v_cap=32, V=1)
    assert int(res.flags.cpu().numpy()[0]) == 0 and res.ivc.shape[-2] == 32
    assert canon(_decode_fold(res, 0)) == canon(exp)
    with pytest.raises(RuntimeError, match="v_cap"):
        _fold(gpu_ctx, maps, 1, 4, 20, V=1)
    maps = _many_values(4, 4, per=12)  # 12 values per register in every input
    exp = O.map_fold_objects(maps)
    assert _max_vals(exp) == 48
    res = _fold(gpu_ctx, maps, 1, 4, 48, v_cap=64, V=12)
    assert int(res.flags.cpu().numpy()[0]) == 0
    assert canon(_decode_fold(res, 0)) == canon(exp)


def test_map_nested_apply_merge_wire_past_8_values(gpu_ctx):
    """States with Vs = 32 value slots: Puts from 20 concurrent writers on one register (the default
    8-slot states flag status bit 4), then merge_batch and the wire form, equal to the oracle."""
    N, K2, A = 4, 4, 24
    base = [O.map_fold_objects([m]) for m in _many_values(1, K2)] * N
    base = [m.copy() for m in base]
    streams, oops = [], []
    for n in range(N):
        ops, oo = [], []
        for i in range(20):
            a = 1 + i  # writer i (actor 1 + i), concurrent with every other
            c = 10 + i
            ops.append(("put", a, c, 0, a, 5, 0, {a: 5}, 1000 * n + i))
            oo.append(MapUp(Dot(a, c), 0, MapUp(Dot(a, 5), 0, MVRegPut(VClock({a: 5}), 1000 * n + i))))
        streams.append(ops)
        oops.append(oo)
    exps = [m.copy() for m in base]
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    assert _max_vals(exps[0]) > 8
    d = O.nested_map_to_dense(base, 1, K2, A, 8)
    z = lambda *s_: torch.zeros(s_, dtype=torch.int64, device="cuda:0")  # noqa: E731
    ivc = z(N, 1, K2, 32, A)
    ivv = z(N, 1, K2, 32)
    ivc[:, :, :, :8] = to_dev(d["ivc"])
    ivv[:, :, :, :8] = to_dev(d["ivv"])
    st8, slots, _ = nested_states(base, 1, K2, A, Dcap=2)
    st = st8._replace(ivc=ivc.contiguous(), ivv=ivv.contiguous())
    enc = cg.map.encode_nested_ops(streams, A, "cuda:0", K2=K2)
    status = cg.map.nested_apply_batch(st, *slots, enc, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    for n in range(N):
        assert canon(decode_states(st, n, [])) == canon(exps[n]), n
    st8, slots8, _ = nested_states(base, 1, K2, A, Dcap=2)  # (fresh: st shares st8's other tensors)
    s8 = cg.map.nested_apply_batch(st8, *slots8, enc, ctx=gpu_ctx).cpu().numpy()
    assert all(x & 16 for x in s8)
    # merge_batch of state 0..1 with 2..3 (Vs = 32 both), then the wire form of the result
    Kw = 1
    slot = lambda: (z(2, 2, A), z(2, 2, Kw), torch.zeros(2, dtype=torch.int32, device="cuda:0"))  # noqa: E731
    me = wire.MapNestedFrames(*[t[:2].contiguous() for t in st], *slot())
    other = wire.MapNestedFrames(*[t[2:].contiguous() for t in st], *slot())
    mst = cg.map.nested_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (mst == 0).all(), mst
    merged = []
    for i in range(2):
        e = exps[i].copy()
        e.merge(exps[2 + i].copy())
        merged.append(e)
        assert canon(decode_states(me, i, [])) == canon(e), i
    r2 = np.random.default_rng(4)
    ad = torch.tensor(np.sort(r2.choice(2**31, size=A, replace=False)), dtype=torch.int32, device="cuda:0")
    kd = torch.tensor([5], dtype=torch.int32, device="cuda:0")
    idd = torch.tensor(np.sort(r2.choice(2**31, size=K2, replace=False)), dtype=torch.int32, device="cuda:0")
    off, data = wire.map_nested_egress(me, ad, kd, idd, ctx=gpu_ctx)
    back, wst = wire.map_nested_ingest(data, off, ad, kd, idd, 2, ctx=gpu_ctx, v_cap=32)
    assert (wst.cpu().numpy() == 0).all()
    for i in range(2):
        assert canon(decode_states(back, i, [])) == canon(merged[i]), i
