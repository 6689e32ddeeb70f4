"""GPU parity: in-place pairwise merge_batch of the causal types (crdt_orswot_merge_batch,
crdt_map_merge_batch) against the oracle's one-pair `merge` (Orswot::merge orswot.rs:81-149,
Map::merge map.rs:140-220 with MVReg::merge mvreg.rs:112-128): N independent
self[i].merge(other[i]) on well-formed op-replay states and on arbitrary states (exact for any
input), plus capacity / invalid-input reporting.  The reference's Orswot KATs also run through
orswot.merge_batch (tests/test_gpu_kat.py, mode "merge_batch")."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host
from orswot_apply_util import arbitrary_case, dense_states, oracle_streams, replay_streams, to_object

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


# ---- Orswot -------------------------------------------------------------------------------------
def orswot_side(states, M, A, Dcap):
    c, e, dc, dm, n = dense_states(states, M, A, Dcap)
    return cg.orswot.OrswotStates(to_dev(c), to_dev(e), to_dev(dc), to_dev(dm), torch.from_numpy(n).cuda())


def orswot_egress(st, N):
    c, e, dc, dm = to_host(st.clock), to_host(st.entries), to_host(st.def_clock), to_host(st.def_members)
    n = st.def_count.cpu().numpy()
    return [to_object(c, e, dc, dm, n, s) for s in range(N)]


def orswot_check(ctx, lhs, rhs, M, A, Dcap=None):
    Dcap = Dcap or max(1, max(len(a.deferred) + len(b.deferred) for a, b in zip(lhs, rhs)))
    me, other = orswot_side(lhs, M, A, Dcap), orswot_side(rhs, M, A, max(1, max(len(b.deferred) for b in rhs)))
    status = cg.orswot.merge_batch(me, other, ctx=ctx).cpu().numpy()
    assert (status == 0).all(), status
    got = orswot_egress(me, len(lhs))
    for i, (a, b) in enumerate(zip(lhs, rhs)):
        exp = a.copy()
        exp.merge(b.copy())
        assert got[i] == exp, i
    return got


@pytest.mark.parametrize("seed,N,M,n_origins,n_ops", [(1, 40, 12, 3, 120), (2, 64, 70, 5, 300), (3, 17, 130, 9, 400)])
def test_orswot_merge_batch_replay(gpu_ctx, seed, N, M, n_origins, n_ops):
    """Well-formed states (op replay at witnesses, test/orswot.rs:33-68 style) merged pairwise."""
    streams = replay_streams(seed, 2 * N, n_origins, M, n_ops)
    states = oracle_streams([O.Orswot() for _ in streams], streams)
    got = orswot_check(gpu_ctx, states[:N], states[N:], M, n_origins)
    assert sum(len(g.deferred) for g in got) > 0 and sum(len(g.entries) for g in got) > 0


@pytest.mark.parametrize("mode", ["", "pocc=0,prows=128"])
@pytest.mark.parametrize("seed,N,M,A", [(11, 50, 40, 16), (12, 33, 9, 3), (13, 20, 200, 65), (14, 30, 300, 64)])
def test_orswot_merge_batch_arbitrary(gpu_ctx, mode, seed, N, M, A):
    """Arbitrary states (deferred removes not dominated, entries beyond the clock after random
    ops): the pairwise kernel is exact without any invariant."""
    ctx = gpu_ctx
    if mode:
        ctx = cg.Context(0)
        ctx.tune(mode)
    states, streams = arbitrary_case(seed, 2 * N, M, A, max_ops=30)
    states = oracle_streams(states, streams)
    orswot_check(ctx, states[:N], states[N:], M, A)


def test_orswot_merge_batch_capacity_and_invalid(gpu_ctx):
    M, A = 8, 4
    a, b = O.Orswot(), O.Orswot()
    a.apply(O.OrswotRm(O.VClock({0: 5}), [1]))
    b.apply(O.OrswotRm(O.VClock({1: 5}), [2]))
    me, other = orswot_side([a, a], M, A, 1), orswot_side([b, b], M, A, 1)
    other.def_count[1] = 7  # invalid on input: that pair is left untouched
    status = cg.orswot.merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert status.tolist() == [1, 4]  # pair 0 needs 2 slots, self has 1
    got = orswot_egress(me, 2)
    assert got[1] == a
    assert got[0].clock == a.clock and len(got[0].deferred) == 1


# pair-join launch forms: the default (one workgroup per CU, 256 member rows), round 2's (no cap,
# 128 rows) and the other row counts / rows-in-flight variants (CRDT_TUNE pocc / prows / pur)
PAIR_MODES = ["", "pocc=0,prows=128", "pocc=2,prows=64", "pocc=2,prows=128,pur=2", "pocc=1,prows=128,pur=4"]


@pytest.mark.parametrize("mode", PAIR_MODES)
def test_orswot_merge_batch_wide(gpu_ctx, mode):
    """A bandwidth-shaped batch (odd A: the 8-byte path; even A: 16-byte path) vs the oracle."""
    ctx = gpu_ctx
    if mode:
        ctx = cg.Context(0)
        ctx.tune(mode)
    for A in (63, 64):
        c, e, off, dcl, dmem = O.gen_orswot(A, 256, 300, A, kmax=20, p_def=0.4)
        states = []
        for s in range(256):
            o = O.Orswot()
            o.clock = O.VClock({a: int(v) for a, v in enumerate(c[s]) if v})
            for m in range(300):
                if e[s, m].any():
                    o.entries[m] = O.VClock({a: int(v) for a, v in enumerate(e[s, m]) if v})
            for d in range(int(off[s]), int(off[s + 1])):
                k = O.VClock({a: int(v) for a, v in enumerate(dcl[d]) if v})
                o.deferred.setdefault(k, set()).update(O.bitmap_members(dmem[d]))
            states.append(o)
        orswot_check(ctx, states[:128], states[128:], 300, A)


# ---- Map<K, MVReg> ------------------------------------------------------------------------------
def map_side(maps, K, A, V, Dcap):
    N = len(maps)
    d = O.map_to_dense(maps, K, A, V)
    Kw = (K + 63) // 64
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    for j, r in enumerate(d["def_row"].astype(np.int64)):
        dcl[r, cnt[r]] = d["def_clock"][j]
        dks[r, cnt[r]] = d["def_keys"][j]
        cnt[r] += 1
    return cg.map.MapStates(to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["vclk"]), to_dev(d["vval"]), to_dev(dcl),
                            to_dev(dks), torch.from_numpy(cnt).cuda())


def map_egress(st, N):
    c, e, vc, vv = to_host(st.clock), to_host(st.ec), to_host(st.vclk), to_host(st.vval)
    dc, dk, n = to_host(st.def_clock), to_host(st.def_keys), st.def_count.cpu().numpy()
    out = []
    for s in range(N):
        deferred = [(dc[s, j], O.bitmap_members(dk[s, j])) for j in range(int(n[s]))]
        out.append((O.dense_to_map(c[s], e[s], vc[s], vv[s], deferred), vc[s], vv[s], e[s]))
    return out


def _canon(m):
    """Map state with each register as its value LIST in Vec order: MVReg's own == asserts that no
    register holds a value twice (mvreg.rs:72), which forgets of arbitrary states can produce
    (two value clocks forgotten to the same clock) in the reference and here alike."""
    return (m.clock, {k: (e.clock, [(tuple(sorted(c.dots.items())), v) for c, v in e.val.vals])
                      for k, e in m.entries.items()}, {k: frozenset(v) for k, v in m.deferred.items()})


def map_check(ctx, lhs, rhs, K, A):
    exp = []
    for a, b in zip(lhs, rhs):
        x = a.copy()
        x.merge(b.copy())
        exp.append(x)
    V1 = max(1, O.max_vals(exp), O.max_vals(lhs))
    V2 = max(1, O.max_vals(rhs))
    Dcap = max(1, max(len(x.deferred) for x in list(lhs) + exp))
    me = map_side(lhs, K, A, V1, Dcap)
    other = map_side(rhs, K, A, V2, max(1, max(len(b.deferred) for b in rhs)))
    status = cg.map.merge_batch(me, other, ctx=ctx).cpu().numpy()
    assert (status == 0).all(), status
    got = map_egress(me, len(lhs))
    for i, ((g, vc, vv, ec), e) in enumerate(zip(got, exp)):
        assert _canon(g) == _canon(e), i
        for k, ent in e.entries.items():  # Vec order: kept own values, then other's added ones
            used = [j for j in range(vc.shape[1]) if vc[k, j].any()]
            assert [int(vv[k, j]) for j in used] == [v for _, v in ent.val.vals], (i, k)
        assert not vc[~ec.any(axis=1)].any()
    return exp


def replay_maps(seed, n, n_origins, K, n_ops):
    from test_gpu_map_apply import oracle_apply, replay_streams as map_replay
    streams = map_replay(seed, n, n_origins, K, n_ops)
    maps, _ = oracle_apply(streams)
    return maps


@pytest.mark.parametrize("seed,N,n_origins,K,n_ops", [(1, 30, 3, 6, 80), (2, 50, 5, 20, 200), (4, 16, 10, 25, 300)])
def test_map_merge_batch_replay(gpu_ctx, seed, N, n_origins, K, n_ops):
    maps = replay_maps(seed, 2 * N, n_origins, K, n_ops)
    exp = map_check(gpu_ctx, maps[:N], maps[N:], K, n_origins)
    assert sum(len(m.entries) for m in exp) > 0


def arbitrary_maps(rng, n, K, A, V, cmax, max_def=3):
    maps = []
    for _ in range(n):
        clock = rng.integers(0, cmax, size=A).astype(np.uint64)
        ec = rng.integers(0, cmax + 1, size=(K, A)).astype(np.uint64)
        ec[rng.random(K) < 0.3] = 0
        vclk = rng.integers(0, cmax + 1, size=(K, V, A)).astype(np.uint64)
        vclk[rng.random((K, V, A)) < 0.5] = 0
        vval = rng.integers(0, 9, size=(K, V)).astype(np.uint64)
        for k in range(K):  # one register never holds two equal clocks (mvreg.rs:72 sanity check)
            for s in range(1, V):
                if any(np.array_equal(vclk[k, s], vclk[k, t]) for t in range(s)):
                    vclk[k, s] = 0
        deferred = []
        for _ in range(int(rng.integers(0, max_def))):
            rm = rng.integers(0, cmax + 2, size=A).astype(np.uint64) * (rng.random(A) < 0.3)
            if rm.any() and not any(np.array_equal(rm, r) for r, _ in deferred):
                deferred.append((rm, set(int(x) for x in rng.choice(K, size=int(rng.integers(1, K + 1)), replace=False))))
        maps.append(O.dense_to_map(clock, ec, vclk, vval, deferred))
    return maps


@pytest.mark.parametrize("reg", ["mpreg=1", "mpreg=1,mpnt=0", "mpreg=1,mppf=1", "mpreg=1,mppf=1,mpbpc=1", "mpreg=2", "mpreg=0"])
@pytest.mark.parametrize("seed,N,K,A,V,cmax", [(21, 40, 5, 3, 2, 4), (22, 25, 9, 33, 2, 3), (23, 16, 4, 70, 1, 3),
                                               (24, 30, 70, 8, 3, 6), (25, 12, 3, 200, 2, 2), (26, 20, 6, 5, 5, 3),
                                               (27, 24, 7, 32, 2, 4), (28, 9, 5, 17, 4, 3), (29, 40, 150, 30, 2, 3)])
def test_map_merge_batch_arbitrary_kernels(gpu_ctx, reg, seed, N, K, A, V, cmax):
    """Arbitrary dense states through each Map key kernel: the sub-wave register kernel (mpreg=1:
    16 / 32 / 64 lanes per key by A; mppf=1 with the next keys' loads in flight; mpbpc=1 one
    workgroup per CU, so a wave walks several keys and the prefetched rows are the ones merged),
    the whole-wave register kernel (mpreg=2, and A > 64 under 1) and the generic one (mpreg=0, and
    self V = 5 under every setting): identical to the oracle."""
    rng = np.random.default_rng(seed)
    maps = arbitrary_maps(rng, N, K, A, V, cmax) + arbitrary_maps(rng, N, K, A, min(V, 2), cmax)
    gpu_ctx.tune(reg)
    try:
        map_check(gpu_ctx, maps[:N], maps[N:], K, A)
    finally:
        gpu_ctx.tune("mpreg=1,mppf=0,mpbpc=64")


def test_map_merge_batch_many_removes(gpu_ctx):
    """More than 64 deferred removes on one pair (the register kernel's remove-bit batch spans
    several waves' worth of lanes)."""
    rng = np.random.default_rng(31)
    maps = arbitrary_maps(rng, 4, 6, 4, 2, 40, max_def=1)
    for m, nd in zip(maps, (40, 3, 35, 70)):
        while len(m.deferred) < nd:
            rm = O.VClock({int(a): int(rng.integers(41, 200)) for a in rng.choice(4, size=2, replace=False)})
            m.deferred.setdefault(rm, set()).update(int(x) for x in rng.choice(6, size=2, replace=False))
    map_check(gpu_ctx, maps[:2], maps[2:], 6, 4)


@pytest.mark.parametrize("seed,N,K,A,V,cmax", [(21, 40, 5, 3, 2, 4), (22, 25, 9, 33, 2, 3), (23, 16, 4, 70, 1, 3),
                                               (24, 30, 70, 8, 3, 6), (25, 12, 3, 200, 2, 2)])
def test_map_merge_batch_arbitrary(gpu_ctx, seed, N, K, A, V, cmax):
    """Arbitrary dense states (any entry / value / deferred clocks): exact without invariants."""
    rng = np.random.default_rng(seed)
    maps = []
    for _ in range(2 * N):
        clock = rng.integers(0, cmax, size=A).astype(np.uint64)
        ec = rng.integers(0, cmax + 1, size=(K, A)).astype(np.uint64)
        ec[rng.random(K) < 0.3] = 0
        vclk = rng.integers(0, cmax + 1, size=(K, V, A)).astype(np.uint64)
        vclk[rng.random((K, V, A)) < 0.5] = 0
        vval = rng.integers(0, 9, size=(K, V)).astype(np.uint64)
        for k in range(K):  # one register never holds two equal clocks (mvreg.rs:72 sanity check)
            for s in range(1, V):
                if any(np.array_equal(vclk[k, s], vclk[k, t]) for t in range(s)):
                    vclk[k, s] = 0
        deferred = []
        for _ in range(int(rng.integers(0, 3))):
            rm = rng.integers(0, cmax + 2, size=A).astype(np.uint64) * (rng.random(A) < 0.3)
            if rm.any() and not any(np.array_equal(rm, r) for r, _ in deferred):
                deferred.append((rm, set(int(x) for x in rng.choice(K, size=int(rng.integers(1, K + 1)), replace=False))))
        maps.append(O.dense_to_map(clock, ec, vclk, vval, deferred))
    map_check(gpu_ctx, maps[:N], maps[N:], K, A)


def test_map_merge_batch_value_overflow(gpu_ctx):
    a, b = O.Map(O.MVReg), O.Map(O.MVReg)
    a.apply(a.update(0, a.get(0).derive_add_ctx(0), lambda r, c: r.write(11, c)))
    b.apply(b.update(0, b.get(0).derive_add_ctx(1), lambda r, c: r.write(22, c)))
    me, other = map_side([a], 1, 2, 1, 1), map_side([b], 1, 2, 1, 1)
    status = cg.map.merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert status[0] == 16  # two concurrent values, one slot: reported
    me = map_side([a], 1, 2, 2, 1)
    assert cg.map.merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()[0] == 0
    x = a.copy()
    x.merge(b.copy())
    assert map_egress(me, 1)[0][0] == x
