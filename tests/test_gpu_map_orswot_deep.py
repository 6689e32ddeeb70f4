"""GPU: Map<K, Orswot<M>> with more than 16 nested deferred removes on one key (round 6).

The reference's Orswot keeps any number of deferred removes (orswot.rs:24, apply_rm :230-250,
merge :81-149); the library's state layouts carry Vd slots per key (crdt_map_orswot_states.Vd /
crdt_map_orswot_out.Vd, 16 by default).  The fold keeps 16 in LDS and re-folds, exactly, the keys
whose list passed 16 with all Vd; the apply, forget, merge_batch and the wire form use all Vd.  Every
case is checked against the oracle's Map / Orswot (a restatement of map.rs / orswot.rs)."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import wire  # noqa: E402


def _deep_maps(rng, R, K, M, A, per=8):
    """R replicas (replica r writes as actor r: A >= R, so no replica's clock dominates another's
    entries) whose keys' Orswots hold up to `per` deferred removes each, clocks from the far future
    on actor 0 (distinct, so a fold unions them: up to R * per on one key)."""
    assert A >= R
    maps = []
    for r in range(R):
        m = O.Map(O.Orswot)
        m.clock = O.VClock({r: 5})
        for k in range(K):
            if rng.random() < 0.9:
                o = O.Orswot()
                o.clock = O.VClock({r: int(rng.integers(1, 4))})
                for mem in range(M):
                    if rng.random() < 0.4:
                        o.entries[mem] = O.VClock({r: int(rng.integers(1, 4))})
                for _ in range(int(rng.integers(1, per + 1))):
                    rm = {0: int(rng.integers(100, 100000))}
                    if rng.random() < 0.5:
                        rm[int(rng.integers(1, A))] = int(rng.integers(1, 3))
                    o.deferred[O.VClock(rm)] = set(int(x) for x in rng.choice(M, size=int(rng.integers(1, min(M, 3) + 1)),
                                                                              replace=False))
                m.entries[k] = O.MapEntry(O.VClock({r: int(rng.integers(1, 5))}), o)
        maps.append(m)
    return maps


def _fold(ctx, maps, K, M, A, G=1, vd_cap="auto", check=True):
    d = O.map_orswot_to_dense(maps, K, M, A)
    R = len(maps) // G
    shp = lambda x: to_dev(x.reshape((G, R) + x.shape[1:]))  # noqa: E731
    Dv = int(d["vd_off"][-1])
    vkw = dict(vd_clock=to_dev(d["vd_clock"]), vd_mem=to_dev(d["vd_members"])) if Dv else {}
    return cg.map.orswot_lub_many(shp(d["clock"]), shp(d["ec"]), shp(d["oc"]), shp(d["ent"]), to_dev(d["vd_off"]),
                                  ctx=ctx, check=check, vd_cap=vd_cap, **vkw)


def _decode(st, n, K, dfr=()):
    c, e, o, m = to_host(st.clock), to_host(st.ec), to_host(st.oc), to_host(st.ent)
    vn, vc, vm = st.vd_n.cpu().numpy(), to_host(st.vd_clock), to_host(st.vd_mem)
    if c.ndim == 1:
        c, e, o, m, vn, vc, vm = c[None], e[None], o[None], m[None], vn[None], vc[None], vm[None]
    mw = (lambda k, i: vm[n, k, i]) if vm.ndim == 4 else (lambda k, i: vm[n, k, i:i + 1])  # noqa: E731
    vd = {k: [(vc[n, k, i], O.bitmap_members(mw(k, i))) for i in range(int(vn[n, k]))] for k in range(K)}
    return O.dense_to_map_orswot(c[n], e[n], o[n], m[n], vd, list(dfr))


def _same(got, exp):
    assert got.clock == exp.clock
    assert got.entries == exp.entries
    assert got.deferred == exp.deferred


def _longest(maps):
    return max(len(e.val.deferred) for x in maps for e in x.entries.values())


@pytest.mark.parametrize("R,K,M,A,seed,vd_cap", [(10, 3, 4, 16, 1, "auto"), (12, 2, 6, 12, 2, 96),
                                                 (6, 3, 70, 8, 3, "auto"), (6, 2, 5, 80, 4, "auto")])
def test_map_orswot_fold_past_16_nested(gpu_ctx, R, K, M, A, seed, vd_cap):
    """The register kernel (M <= 32, A <= 64) and the wide kernel (M = 70, A = 80) as the first pass;
    the keys past 16 re-folded with all Vd slots: equal to the oracle's left fold."""
    rng = np.random.default_rng(seed)
    maps = _deep_maps(rng, R, K, M, A)
    exp = O.map_fold_objects(maps)
    assert _longest([exp]) > 16
    res = _fold(gpu_ctx, maps, K, M, A, vd_cap=vd_cap)
    assert res.vd_clock.shape[-2] >= _longest([exp])
    assert int(res.flags.cpu().numpy()[0]) == 0
    _same(_decode(res, 0, K), exp)


def test_map_orswot_fold_groups_mixed_depths(gpu_ctx):
    """G = 4 groups, two with keys past 16 nested removes and two within: only the deep keys re-fold,
    every group equal to its own fold."""
    K, M, A, R = 3, 5, 8, 8
    rng = np.random.default_rng(7)
    parts = [_deep_maps(rng, R, K, M, A, per=8 if g % 2 == 0 else 1) for g in range(4)]
    res = _fold(gpu_ctx, [m for p in parts for m in p], K, M, A, G=4, vd_cap=80)
    for g in range(4):
        exp = O.map_fold_objects(parts[g])
        _same(_decode(res, g, K), exp)
    assert _longest([O.map_fold_objects(parts[0])]) > 16 >= _longest([O.map_fold_objects(parts[1])])


def test_map_orswot_fold_vd_cap_16_flags(gpu_ctx):
    """The default 16 slots on a fold that needs more: flags bit 4, raised by check=True (never a
    silently truncated state)."""
    rng = np.random.default_rng(5)
    maps = _deep_maps(rng, 10, 2, 4, 10)
    with pytest.raises(RuntimeError, match="vd_cap"):
        _fold(gpu_ctx, maps, 2, 4, 10, vd_cap=16)
    res = _fold(gpu_ctx, maps, 2, 4, 10, vd_cap=16, check=False)
    assert int(res.flags.cpu().numpy()[0]) & 16


def _slots(N, Dcap, A, K):
    z = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    return z(N, Dcap, A), z(N, Dcap, (K + 63) // 64), torch.zeros(N, dtype=torch.int32, device="cuda:0")


@pytest.mark.parametrize("M,A", [(4, 8), (70, 8)])
def test_map_orswot_apply_past_16_nested(gpu_ctx, M, A):
    """Orswot Rms from the far future on one key, 40 per state, on states with Vd = 64 slots: the
    nested list grows past 16 (masks of all 64 in LDS) and later Adds re-apply every one of them."""
    N, K, T = 8, 3, 60
    rng = np.random.default_rng(11 + M)
    base = _deep_maps(rng, N, K, M, A, per=1)  # (no Map-level removes)
    exps = [O.map_fold_objects([m]) for m in base]
    d = O.map_orswot_to_dense(base, K, M, A)
    shp = lambda x: to_dev(x.reshape((N, 1) + x.shape[1:]))  # noqa: E731
    Dv = int(d["vd_off"][-1])
    vkw = dict(vd_clock=to_dev(d["vd_clock"]), vd_mem=to_dev(d["vd_members"])) if Dv else {}
    assert d["def_row"].shape[0] == 0
    res = cg.map.orswot_lub_many(shp(d["clock"]), shp(d["ec"]), shp(d["oc"]), shp(d["ent"]), to_dev(d["vd_off"]),
                                 ctx=gpu_ctx, vd_cap=64, **vkw)
    streams, oops = [], []
    for x in exps:
        clk = {a: x.clock.get(a) for a in range(A)}
        ops, oo = [], []
        for i in range(T):
            a = int(rng.integers(A))
            clk[a] += 1
            ms = sorted(set(int(z) for z in rng.choice(M, size=int(rng.integers(1, 3)), replace=False)))
            if i % 3 != 2:  # an Orswot Rm from the future on key 0
                row = {0: 1000 + i, int(rng.integers(1, A)): 1}
                ops.append(("orm", a, clk[a], 0, row, ms))
                oo.append(O.MapUp(O.Dot(a, clk[a]), 0, O.OrswotRm(O.VClock(row), ms)))
            else:  # an Add on key 0 (re-applies every nested remove) or another key
                k = 0 if rng.random() < 0.7 else int(rng.integers(1, K))
                va = int(rng.integers(1, A))
                ops.append(("add", a, clk[a], k, va, 50 + i, ms))
                oo.append(O.MapUp(O.Dot(a, clk[a]), k, O.OrswotAdd(O.Dot(va, 50 + i), ms)))
        streams.append(ops)
        oops.append(oo)
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    assert 16 < _longest(exps) <= 64
    tdc, tdk, tcnt = _slots(N, 4, A, K)
    ops = cg.map.encode_orswot_map_ops(streams, A, "cuda:0")
    status = cg.map.orswot_apply_batch(res, tdc, tdk, tcnt, ops, ctx=gpu_ctx).cpu().numpy()
    for n in range(N):
        assert status[n] == 0, (n, status[n])
        _same(_decode(res, n, K), exps[n])
    # the same stream with 16 slots flags the overflow (status bit 0), never past the slots
    res16 = cg.map.orswot_lub_many(shp(d["clock"]), shp(d["ec"]), shp(d["oc"]), shp(d["ent"]), to_dev(d["vd_off"]),
                                   ctx=gpu_ctx, **vkw)
    st16 = cg.map.orswot_apply_batch(res16, *_slots(N, 4, A, K), ops, ctx=gpu_ctx).cpu().numpy()
    assert all(s & 1 for s in st16)
    assert int(res16.vd_n.max()) <= 16


def test_map_orswot_forget_merge_wire_past_16_nested(gpu_ctx):
    """Deep states (Vd = 128: the merged lists reach ~100) through forget, merge_batch and the wire
    form, each equal to the oracle."""
    K, M, A, R, N = 3, 5, 9, 9, 4
    rng = np.random.default_rng(21)
    groups = [_deep_maps(rng, R, K, M, A) for _ in range(2 * N)]
    folds = [O.map_fold_objects(g) for g in groups]
    assert _longest(folds) > 16
    res = _fold(gpu_ctx, [m for g in groups for m in g], K, M, A, G=2 * N, vd_cap=128)
    Dc = 2
    me = wire.MapOrswotFrames(*[t[:N].contiguous() for t in res[:7]], *_slots(N, Dc, A, K))
    other = wire.MapOrswotFrames(*[t[N:].contiguous() for t in res[:7]], *_slots(N, Dc, A, K))
    # wire round trip of self (Vd slots carried through ingest)
    rng2 = np.random.default_rng(3)
    aids = np.sort(rng2.choice(2**31, size=A, replace=False)).astype(np.int64)
    kids = np.sort(rng2.choice(2**31, size=K, replace=False)).astype(np.int64)
    mids = np.sort(rng2.choice(2**62, size=M, replace=False)).astype(np.int64)
    ad = torch.tensor(aids, dtype=torch.int32, device="cuda:0")
    kd = torch.tensor(kids, dtype=torch.int32, device="cuda:0")
    md = torch.tensor(mids, dtype=torch.int64, device="cuda:0")
    off, data = wire.map_orswot_egress(me, ad, kd, md, ctx=gpu_ctx)
    back, st = wire.map_orswot_ingest(data, off, ad, kd, md, Dc, ctx=gpu_ctx, vd_cap=128)
    assert (st.cpu().numpy() == 0).all()
    for i in range(N):
        _same(_decode(back, i, K), folds[i])
    # merge_batch: self[i].merge(other[i])
    status = cg.map.orswot_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    for i in range(N):
        exp = folds[i].copy()
        exp.merge(folds[N + i].copy())
        _same(_decode(me, i, K), exp)
    # forget by a clock that forgets about half the removes (actor 0 below 50,000)
    y = torch.zeros(A, dtype=torch.int64, device="cuda:0")
    y[0] = 50000
    cg.map.orswot_forget_batch(me, y, ctx=gpu_ctx)
    for i in range(N):
        exp = folds[i].copy()
        exp.merge(folds[N + i].copy())
        exp.forget(O.VClock({0: 50000}))
        _same(_decode(me, i, K), exp)


def _many_live(R, K, mk_val, per=8):
    """R replicas (actor r) each holding `per` Map-level removes from the far future on actor 0 that
    name key 0 (distinct clocks: a fold keeps all R * per live on key 0, past the 256 the first pass
    holds)."""
    maps = []
    for r in range(R):
        m = O.Map(mk_val)
        m.clock = O.VClock({r: 5})
        for k in range(K):
            m.entries[k] = O.MapEntry(O.VClock({r: 2 + k % 2}), mk_val(r, k))
        for i in range(per):
            m.deferred[O.VClock({0: 1000 + per * r + i})] = {0} if i % 3 else {0, K - 1}
        maps.append(m)
    return maps


def test_map_orswot_fold_past_256_live_removes(gpu_ctx):
    """320 live Map-level removes naming one key (flags bit 3 before round 6): the deep pass holds the
    group's whole remove list; equal to the oracle's fold, Map-level survivors included."""
    from test_gpu_map_orswot import _got_maps, _run

    def val(r, k):
        o = O.Orswot()
        o.clock = O.VClock({r: 2})
        o.entries[k % 3] = O.VClock({r: 1 + k % 2})
        return o
    R, K, M, A = 40, 3, 3, 40
    maps = _many_live(R, K, lambda *a: val(*a) if a else O.Orswot())
    exp = O.map_fold_objects(maps)
    assert len(exp.deferred) > 256
    d = O.map_orswot_to_dense(maps, K, M, A)
    res, kw = _run(gpu_ctx, d)
    assert int(res.flags.cpu().numpy()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)
