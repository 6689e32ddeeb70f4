"""GPU parity: Map<K, Orswot<M>> lub_many (crdt_map_orswot_lub_many, round 4) against the oracle's
left fold of Map::merge (map.rs:140-220) with Orswot::merge / forget (orswot.rs:81-183) as the
value's: the reference's merge_error KAT (map.rs:435-494) folded both ways, op-replay replicas
whose nested sets add and remove members with contexts that leave deferred removes at both
levels, arbitrary dense states, several groups with a CSR pool, and an empty fold."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _run(ctx, d, G=1, off=None):
    R = d["clock"].shape[0] // G
    shp = lambda x: x.reshape((G, R) + x.shape[1:])  # noqa: E731
    D = d["def_row"].shape[0]
    kw = {}
    if D:
        kw = dict(def_off=off if off is not None else [0, D],
                  def_row=torch.from_numpy(np.asarray(d["def_row"], np.int64).astype(np.int32)).cuda(),
                  def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"]))
    Dv = int(d["vd_off"][-1])
    vkw = dict(vd_clock=to_dev(d["vd_clock"]), vd_mem=to_dev(d["vd_members"])) if Dv else {}
    res = cg.map.orswot_lub_many(to_dev(shp(d["clock"])), to_dev(shp(d["ec"])), to_dev(shp(d["oc"])),
                                 to_dev(shp(d["ent"])), to_dev(d["vd_off"]), ctx=ctx, **vkw, **kw)
    return res, kw


def _got_maps(res, kw, G):
    out = []
    c, e, o, m = to_host(res.clock), to_host(res.ec), to_host(res.oc), to_host(res.ent)
    vn = res.vd_n.cpu().numpy().reshape(G, -1)
    vc, vm = to_host(res.vd_clock), to_host(res.vd_mem)
    if c.ndim == 1:
        c, e, o, m, vc, vm = c[None], e[None], o[None], m[None], vc[None], vm[None]
    for g in range(G):
        dset = set()
        if kw:
            off = kw["def_off"]
            dset = cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys, int(off[g]), int(off[g + 1]))
        mw = (lambda k, i: vm[g, k, i]) if vm.ndim == 4 else (lambda k, i: vm[g, k, i:i + 1])  # noqa: E731
        vd = {k: [(vc[g, k, i], O.bitmap_members(mw(k, i))) for i in range(int(vn[g, k]))]
              for k in range(e.shape[1])}
        out.append(O.dense_to_map_orswot(c[g], e[g], o[g], m[g], vd,
                                         [(np.array(rm, np.uint64), ks) for rm, ks in dset]))
    return out


def _same(got, exp):
    assert got.clock == exp.clock
    assert got.entries == exp.entries
    assert got.deferred == exp.deferred


def _intern(maps):
    """Dense indices for the KAT's u8 actors / keys / members."""
    acts, keys, mems = set(), set(), set()
    for m in maps:
        acts |= set(m.clock.dots)
        for k, e in m.entries.items():
            keys.add(k)
            acts |= set(e.clock.dots) | set(e.val.clock.dots)
            for mem, mc in e.val.entries.items():
                mems.add(mem)
                acts |= set(mc.dots)
    ai = {a: i for i, a in enumerate(sorted(acts))}
    ki = {k: i for i, k in enumerate(sorted(keys))}
    mi = {x: i for i, x in enumerate(sorted(mems))}

    def vc(c):
        return O.VClock({ai[a]: n for a, n in c.dots.items()})

    out = []
    for m in maps:
        n = O.Map(O.Orswot)
        n.clock = vc(m.clock)
        for k, e in m.entries.items():
            o = O.Orswot()
            o.clock = vc(e.val.clock)
            o.entries = {mi[x]: vc(c) for x, c in e.val.entries.items()}
            n.entries[ki[k]] = O.MapEntry(vc(e.clock), o)
        out.append(n)
    return out, len(ai), len(ki), len(mi)


def test_map_orswot_merge_error_kat(gpu_ctx):
    """map.rs:435-494: m1 (clock {75: 1}) merged with m2 (key 101 -> Orswot {1: {75: 1}, 2: {93: 1}})
    keeps only member 2 under entry clock {93: 1}; folded as [m1, m2] and as [m2, m1]."""
    def vc(*ds):
        return O.VClock({a: c for a, c in ds})

    m1 = O.Map(O.Orswot)
    m1.clock = vc((75, 1))
    m2 = O.Map(O.Orswot)
    m2.clock = vc((75, 1), (93, 1))
    o = O.Orswot()
    o.clock = vc((75, 1), (93, 1))
    o.entries = {1: vc((75, 1)), 2: vc((93, 1))}
    m2.entries = {101: O.MapEntry(vc((75, 1), (93, 1)), o)}
    (d1, d2), A, K, M = _intern([m1, m2])
    for maps in ([d1, d2], [d2, d1]):
        exp = O.map_fold_objects(maps)
        d = O.map_orswot_to_dense(maps, K, M, A)
        res, kw = _run(gpu_ctx, d)
        got = _got_maps(res, kw, 1)[0]
        _same(got, exp)
    # the KAT's expected state, in interned form: actor 93 -> 1, member 2 -> 1
    assert got.entries[0].clock == O.VClock({1: 1})
    assert got.entries[0].val.entries == {1: O.VClock({1: 1})}


@pytest.mark.parametrize("seed,R,K,M,A", [(1, 40, 4, 5, 4), (2, 60, 6, 8, 5), (3, 30, 3, 12, 6),
                                           (4, 80, 8, 3, 8), (5, 50, 5, 32, 3)])
def test_map_orswot_op_replay(gpu_ctx, seed, R, K, M, A):
    maps = O.map_orswot_objects(R, K, M, A, seed=seed, steps=7 * R)
    exp = O.map_fold_objects(maps)
    d = O.map_orswot_to_dense(maps, K, M, A)
    res, kw = _run(gpu_ctx, d)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


def test_map_orswot_nested_deferred_survive(gpu_ctx):
    """Enough op-replay histories that some folds end with nested deferred removes."""
    n = 0
    for seed in range(10, 22):
        maps = O.map_orswot_objects(30, 3, 6, 4, seed=seed, steps=220, p_vrm=0.5)
        exp = O.map_fold_objects(maps)
        n += sum(len(e.val.deferred) for e in exp.entries.values())
        d = O.map_orswot_to_dense(maps, 3, 6, 4)
        res, kw = _run(gpu_ctx, d)
        _same(_got_maps(res, kw, 1)[0], exp)
    assert n > 0


def _arbitrary(rng, R, K, M, A, cmax):
    maps = []
    for _ in range(R):
        m = O.Map(O.Orswot)
        m.clock = O.VClock({a: int(x) for a, x in enumerate(rng.integers(0, cmax + 1, A)) if x})
        for k in range(K):
            if rng.random() < 0.6:
                ec = {a: int(x) for a, x in enumerate(rng.integers(0, cmax + 2, A)) if x and rng.random() < 0.5}
                if not ec:
                    continue
                o = O.Orswot()
                o.clock = O.VClock({a: int(x) for a, x in enumerate(rng.integers(0, cmax + 2, A)) if x})
                for mem in range(M):
                    if rng.random() < 0.5:
                        dots = {a: int(x) for a, x in enumerate(rng.integers(0, cmax + 2, A)) if x and rng.random() < 0.5}
                        if dots:
                            o.entries[mem] = O.VClock(dots)
                for _ in range(int(rng.integers(0, 3))):
                    rm = {a: int(x) for a, x in enumerate(rng.integers(0, cmax + 3, A)) if x and rng.random() < 0.4}
                    if rm:
                        o.deferred[O.VClock(rm)] = set(int(x) for x in rng.choice(M, size=int(rng.integers(1, M + 1)),
                                                                                    replace=False))
                m.entries[k] = O.MapEntry(O.VClock(ec), o)
        for _ in range(int(rng.integers(0, 2))):
            rm = {a: int(x) for a, x in enumerate(rng.integers(0, cmax + 3, A)) if x and rng.random() < 0.4}
            if rm:
                m.deferred[O.VClock(rm)] = set(int(x) for x in rng.choice(K, size=int(rng.integers(1, K + 1)),
                                                                            replace=False))
        maps.append(m)
    return maps


@pytest.mark.parametrize("seed,R,K,M,A,cmax", [(21, 20, 3, 4, 5, 3), (22, 30, 4, 6, 3, 4), (23, 12, 2, 9, 64, 3),
                                                (24, 25, 5, 2, 7, 2)])
def test_map_orswot_arbitrary(gpu_ctx, seed, R, K, M, A, cmax):
    rng = np.random.default_rng(seed)
    maps = _arbitrary(rng, R, K, M, A, cmax)
    exp = O.map_fold_objects(maps)
    if any(len(e.val.deferred) > cg.map.VD_CAP for e in exp.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    d = O.map_orswot_to_dense(maps, K, M, A)
    res, kw = _run(gpu_ctx, d)
    _same(_got_maps(res, kw, 1)[0], exp)


def test_map_orswot_groups(gpu_ctx):
    """G = 3 groups of one launch: the value CSR spans the groups, the Map pool has CSR offsets."""
    G, R, K, M, A = 3, 25, 4, 5, 4
    parts = [O.map_orswot_objects(R, K, M, A, seed=60 + g, steps=180) for g in range(G)]
    allm = [m for p in parts for m in p]
    d = O.map_orswot_to_dense(allm, K, M, A)
    d["def_row"] = d["def_row"] % R  # (rows within the group)
    off = [0]
    for p in parts:
        off.append(off[-1] + sum(len(m.deferred) for m in p))
    res, kw = _run(gpu_ctx, d, G=G, off=off)
    got = _got_maps(res, kw, G)
    for g in range(G):
        _same(got[g], O.map_fold_objects(parts[g]))


def test_map_orswot_empty(gpu_ctx):
    """R = 0 folds to Map::new()."""
    z = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    res = cg.map.orswot_lub_many(z(2, 0, 4), z(2, 0, 3, 4), z(2, 0, 3, 4), z(2, 0, 3, 5, 4), z(1), ctx=gpu_ctx)
    assert not to_host(res.clock).any() and not to_host(res.ec).any() and not to_host(res.ent).any()
    assert not res.vd_n.cpu().numpy().any()


def test_map_orswot_vd_off_validation(gpu_ctx):
    """vd_off must be int64 / uint64, start at 0, never decrease and end at the rows of
    vd_clock; a malformed CSR is reported (flags bit 5 -> ValueError), never read past its rows."""
    maps = O.map_orswot_objects(20, 3, 5, 4, seed=3, steps=160, p_vrm=0.5)
    d = O.map_orswot_to_dense(maps, 3, 5, 4)
    Dv = int(d["vd_off"][-1])
    assert Dv >= 2
    args = lambda: (to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["oc"]), to_dev(d["ent"]))  # noqa: E731
    vkw = dict(vd_clock=to_dev(d["vd_clock"]), vd_mem=to_dev(d["vd_members"]))
    off32 = torch.from_numpy(np.asarray(d["vd_off"], np.int64).astype(np.int32)).cuda()
    with pytest.raises(ValueError, match="int64"):
        cg.map.orswot_lub_many(*args(), off32, ctx=gpu_ctx, **vkw)
    bad = np.asarray(d["vd_off"], np.uint64).copy()
    i = int(np.flatnonzero(np.diff(bad.astype(np.int64)) > 0)[0]) + 1  # an entry that can be lowered
    bad[i] = bad[i - 1] + np.uint64(Dv + 5)  # then the next entry decreases
    with pytest.raises(ValueError, match="vd_off invalid"):
        cg.map.orswot_lub_many(*args(), to_dev(bad), ctx=gpu_ctx, **vkw)
    extra = dict(vd_clock=to_dev(np.concatenate([d["vd_clock"], d["vd_clock"][:1]])),
                 vd_mem=to_dev(np.concatenate([d["vd_members"], d["vd_members"][:1]])))
    with pytest.raises(ValueError, match="vd_off invalid"):  # last entry != rows of vd_clock
        cg.map.orswot_lub_many(*args(), to_dev(d["vd_off"]), ctx=gpu_ctx, **extra)
    res = cg.map.orswot_lub_many(*args(), to_dev(d["vd_off"]), ctx=gpu_ctx, **vkw)  # the valid CSR still folds
    assert int(res.flags.cpu()[0]) == 0


@pytest.mark.parametrize("M,R", [(4, 16), (4, 17), (4, 24), (8, 8), (8, 9), (8, 12), (32, 4), (32, 5), (32, 6)])
def test_map_orswot_ring_block_boundaries(gpu_ctx, M, R):
    """the register ring runs unclamped blocks while r0 + 2*DEPTH < R and clamped ones after;
    R = 2*DEPTH, 2*DEPTH + 1 and 3*DEPTH for DEPTH = 8 / 4 / 2 (M <= 4 / <= 8 / <= 32)."""
    maps = O.map_orswot_objects(R, 3, M, 4, seed=100 + R + M, steps=12 * R, p_vrm=0.4)
    exp = O.map_fold_objects(maps)
    d = O.map_orswot_to_dense(maps, 3, M, 4)
    res, kw = _run(gpu_ctx, d)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


def test_map_orswot_dominated_nested_removes_not_held(gpu_ctx):
    """a replica's nested removes already covered by our Orswot clock (rm <= oc) are applied
    and never deferred (orswot.rs:230-238), so 20 of them do not count toward the 16-remove capacity."""
    m0 = O.Map(O.Orswot)
    m0.clock = O.VClock({0: 5, 1: 5})
    o0 = O.Orswot()
    o0.clock = O.VClock({0: 5, 1: 5})
    o0.entries = {0: O.VClock({0: 5}), 1: O.VClock({1: 3})}
    m0.entries[0] = O.MapEntry(O.VClock({0: 5}), o0)
    m1 = O.Map(O.Orswot)
    m1.clock = O.VClock({0: 5, 2: 1})
    o1 = O.Orswot()
    o1.clock = O.VClock({0: 5, 2: 1})
    o1.entries = {0: O.VClock({0: 5}), 2: O.VClock({2: 1})}
    n = 0
    for a in range(1, 6):
        for b in range(1, 5):
            if n < 20:
                o1.deferred[O.VClock({0: a, 1: b})] = {1 + (n % 2)}
                n += 1
    m1.entries[0] = O.MapEntry(O.VClock({0: 5, 2: 1}), o1)
    maps = [m0, m1]
    exp = O.map_fold_objects(maps)
    d = O.map_orswot_to_dense(maps, 1, 3, 3)
    res, kw = _run(gpu_ctx, d)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.fixture(params=["mocs=1", "", "mowide=1"])
def moctx(request):
    """The whole-chunk skip (mocs=1, opt-in; A = 32 / 16 / 8 with up to 4 members, round 5), the
    default register ring and the wide kernel (mowide=1; the one past A = 64 / M = 32)."""
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    if request.param:
        ctx.tune(request.param)
    yield ctx
    ctx.close()


@pytest.mark.parametrize("seed,R,K,M,A", [(41, 120, 3, 4, 32), (42, 150, 4, 3, 16), (43, 100, 3, 4, 8),
                                           (44, 90, 2, 2, 32)])
def test_map_orswot_chunk_skip_op_replay(moctx, seed, R, K, M, A):
    """The chunk-skip shapes over long op-replay folds: nested removes inside chunks (exact), chunks
    skipped in between, a partial last chunk."""
    maps = O.map_orswot_objects(R, K, M, A, seed=seed, steps=6 * R, p_vrm=0.4)
    exp = O.map_fold_objects(maps)
    d = O.map_orswot_to_dense(maps, K, M, A)
    res, kw = _run(moctx, d)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.mark.parametrize("seed,R,A,cmax", [(56, 40, 16, 3), (66, 32, 32, 2), (64, 24, 32, 3), (53, 80, 8, 4),
                                            (58, 80, 8, 3)])
def test_map_orswot_chunk_skip_arbitrary(moctx, seed, R, A, cmax):
    """Arbitrary states (nested removes never applied to their rows, entry dots above clocks) at the
    chunk-skip shapes: a replica's Orswot taken as it comes leaves the state un-normalized, which the
    skip must not assume.  (Parameters chosen so that no fold state holds more than 11 nested removes,
    well inside the kernel's 16: random rm clocks over many actors are rarely dominated.)"""
    rng = np.random.default_rng(seed)
    maps = _arbitrary(rng, R, 3, 4, A, cmax)
    exp = O.map_fold_objects(maps)
    if any(len(e.val.deferred) > cg.map.VD_CAP for e in exp.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    d = O.map_orswot_to_dense(maps, 3, 4, A)
    res, kw = _run(moctx, d)
    _same(_got_maps(res, kw, 1)[0], exp)


def test_map_orswot_chunk_skip_steady_state(moctx):
    """Replicas repeating one folded state with growing clocks (every chunk skippable), then a late
    replica with new dots: the skipped chunks merge only their clocks."""
    A, K, M, R = 32, 2, 4, 160
    base = O.map_orswot_objects(10, K, M, A, seed=61, steps=100, p_vrm=0.3)
    fold = O.map_fold_objects(base)
    maps = []
    for r in range(R):
        m = fold.copy()
        m.clock.apply(O.Dot(r % A, fold.clock.get(r % A) + 1 + r // A))
        maps.append(m)
    late = O.map_orswot_objects(4, K, M, A, seed=62, steps=60, p_vrm=0.5)
    maps[130] = late[-1]
    exp = O.map_fold_objects(maps)
    d = O.map_orswot_to_dense(maps, K, M, A)
    res, kw = _run(moctx, d)
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.mark.parametrize("R1,R2,late", [(200, 2400, 2300), (120, 500, 400), (64, 2060, 2100)])
def test_map_orswot_chunk_mode_switch(moctx, R1, R2, late):
    """The chunk-skip mode's exits: R1 op-replay replicas (each a different view of the history: chunks
    fail, and the wave leaves for kMoRingSpan = 2048 register-ring steps, which end inside the fold
    or at its last replica), then R2 replicas repeating the fold so far (nested removes held) with
    growing clocks (chunks pass again once the ring span is over), one late replica with new dots,
    and a partial last chunk."""
    A, K, M = 32, 2, 4
    first = O.map_orswot_objects(R1, K, M, A, seed=R1, steps=6 * R1, p_vrm=0.4)
    fold = O.map_fold_objects(first)
    maps = list(first)
    for r in range(R2):
        m = fold.copy()
        m.clock.apply(O.Dot(r % A, fold.clock.get(r % A) + 1 + r // A))
        maps.append(m)
    if late < len(maps):
        maps[late] = O.map_orswot_objects(4, K, M, A, seed=63, steps=60, p_vrm=0.5)[-1]
    maps.append(fold.copy())
    exp = O.map_fold_objects(maps)
    d = O.map_orswot_to_dense(maps, K, M, A)
    res, kw = _run(moctx, d)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.mark.parametrize("seed,R,K,M,A", [(71, 40, 3, 40, 100), (72, 30, 2, 70, 64), (73, 24, 2, 6, 300),
                                           (74, 20, 2, 130, 70), (75, 12, 2, 3, 1024)])
def test_map_orswot_wide_shapes(gpu_ctx, seed, R, K, M, A):
    """Past the register kernel's limits (A > 64 actors: 2 / 8 / 16 words per lane; M > 32 members,
    past 64: multi-word nested member masks), op-replay folds with deferred removes at both levels."""
    maps = O.map_orswot_objects(R, K, M, A, seed=seed, steps=8 * R, p_vrm=0.4)
    exp = O.map_fold_objects(maps)
    d = O.map_orswot_to_dense(maps, K, M, A)
    res, kw = _run(gpu_ctx, d)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


def test_map_orswot_wide_grouped_arbitrary(gpu_ctx):
    """Arbitrary states at A = 96 in 3 groups of one launch (the group offsets of every row, the value
    CSR spanning the groups, the Map pool's CSR offsets) through the wide kernel."""
    rng = np.random.default_rng(77)
    G, R, K, M, A = 3, 16, 3, 4, 96
    parts = [_arbitrary(rng, R, K, M, A, 3) for _ in range(G)]
    exps = [O.map_fold_objects(p) for p in parts]
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in exps for e in x.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    d = O.map_orswot_to_dense([m for p in parts for m in p], K, M, A)
    d["def_row"] = d["def_row"] % R  # (rows within the group)
    off = [0]
    for p in parts:
        off.append(off[-1] + sum(len(m.deferred) for m in p))
    res, kw = _run(gpu_ctx, d, G=G, off=off)
    for g, got in enumerate(_got_maps(res, kw, G)):
        _same(got, exps[g])


# ---- the 4-step ring at >= 2,048 key waves (round 6: two waves per SIMD) ------------------------------
def test_map_orswot_shallow_ring_many_groups(gpu_ctx):
    """G = 512 groups x K = 4 keys (2,048 key waves: the library's 4-step-ring instance), op-replay replicas
    with deferred removes at both levels, 8 per group: every group equal to its own left fold."""
    G, R, K, M, A = 512, 8, 4, 4, 6
    maps = O.map_orswot_objects(G * R, K, M, A, seed=99, steps=3 * G * R, p_vrm=0.5)
    d = O.map_orswot_to_dense(maps, K, M, A)
    d["def_row"] = d["def_row"] % R
    off = [0]
    for g in range(G):
        off.append(off[-1] + sum(len(m.deferred) for m in maps[g * R:(g + 1) * R]))
    exps = [O.map_fold_objects(maps[g * R:(g + 1) * R]) for g in range(G)]
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in exps for e in x.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    res, kw = _run(gpu_ctx, d, G=G, off=off if off[-1] else None)
    got = _got_maps(res, kw, G)
    for g in range(G):
        _same(got[g], exps[g])
