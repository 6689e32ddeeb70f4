"""GPU parity: Map<K, MVReg<u64>> lub_many vs the oracle's reference fold (C++ twin over
map-based states, oracle/ref_fold.cpp; itself pinned by the reference's map/mvreg tests and
cross-checked with the Python twin in tests/test_oracle_map_dense.py).  Bit-exact on entry
clocks, value clocks, values (in Vec order), value counts and surviving deferred removes."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402

# Staging paths of the fold kernel (results must not depend on them): LDS-DMA ring with
# 16-replica chunks in 2 slots or 8-replica chunks in 4 slots (taken where A is even, V <= 2 and
# the state fits 4 values), and register staging (every shape); the speculative scan with two
# actors per 16-byte LDS read (mscan2=1, even A; off by default: no faster), the threshold scan
# (mscan3=1, the default of the LDS-DMA ring) and the non-temporal step-image loads (mnt=1, off by
# default); and the register-staged whole-chunk skip (mrs=1, the default where A <= 32 on the
# LDS-DMA shapes), also with the scan off (mspec=0: every chunk handed to the exact loop); and at
# A = 32, V = 2, K % 4 == 0 the RS path with four key waves sharing each chunk's clock rows (msh=1,
# opt-in: less traffic, slower); and at A = 32, V = 2 the RS path with two waves per key, each testing
# 8 steps of every chunk (mst=1, ST) or one (mst=0).
MODES = ["mglds=1,mrs=1", "mglds=1,mrs=1,mspec=0", "mglds=1,mrs=1,msh=1", "mglds=1,mrs=1,mst=0", "mglds=1,mrs=1,mst=1",
         "mglds=1,mrs=0,mchunk=16,mring=2,mscan3=1,mnt=0", "mglds=1,mrs=0,mchunk=8,mring=4,mscan3=1,mnt=0",
         "mglds=0,mscan2=0,mnt=0", "mglds=1,mrs=0,mchunk=16,mring=2,mscan3=0,mscan2=0,mnt=0",
         "mglds=1,mrs=0,mchunk=16,mring=2,mscan3=0,mscan2=1,mnt=1", "mglds=0,mscan2=1,mnt=0"]


@pytest.fixture(scope="module", params=MODES)
def mctx(request):
    import torch
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    ctx.tune(request.param)
    return ctx


def _gpu(gpu_ctx, d, vout, groups=None):
    """d: dense dict of one group (or stacked when groups = list of per-group D counts)."""
    D = d["def_clock"].shape[0]
    kw = {}
    if D:
        G = 1 if groups is None else len(groups)
        off = [0] + list(np.cumsum(groups if groups is not None else [D]))
        kw = dict(def_off=off,
                  def_row=torch.from_numpy(np.asarray(d["def_row"], np.int64).astype(np.int32)).cuda(),
                  def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"]))
    res = cg.map.lub_many(to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["vclk"]), to_dev(d["vval"]),
                          vout=vout, ctx=gpu_ctx, **kw)
    return res, kw


def _check(gpu_ctx, d, vout):
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                     d["def_keys"], vout)
    res, kw = _gpu(gpu_ctx, d, vout)
    np.testing.assert_array_equal(to_host(res.clock), exp[0])
    np.testing.assert_array_equal(to_host(res.ec), exp[1])
    np.testing.assert_array_equal(to_host(res.vclk), exp[2])
    np.testing.assert_array_equal(to_host(res.vval), exp[3])
    np.testing.assert_array_equal(res.nval.cpu().numpy(), exp[4])
    got = cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys) if kw else set()
    assert got == exp[5]
    return exp


@pytest.mark.parametrize("seed", range(24))
def test_map_lub_many_op_replay(mctx, seed):
    rng = np.random.default_rng(seed)
    K, A = int(rng.integers(1, 70)), int(rng.integers(1, 9))
    R = int(rng.integers(1, 40))
    p_rm = float(rng.choice([0.15, 0.3, 0.45]))
    maps = O.gen_map_replicas(seed, R, K, A, steps=int(rng.integers(20, 300)), p_rm=p_rm, p_up=0.7 - p_rm)
    V = O.max_vals(maps)
    d = O.map_to_dense(maps, K, A, V)
    vout = max(4, O.max_vals([O.map_fold_objects(maps)]))
    _check(mctx, d, vout)


def _random_dense(rng, R, K, A, V, cmax, D=None, keys_per_rm=None):
    # replica clocks mostly below the entry clocks, so that entries survive the fold
    clock = rng.integers(0, max(2, cmax // 2), size=(R, A)).astype(np.uint64)
    ec = rng.integers(0, cmax, size=(R, K, A)).astype(np.uint64)
    ec[rng.random((R, K)) < 0.3] = 0
    vclk = rng.integers(0, cmax, size=(R, K, V, A)).astype(np.uint64)
    vclk[rng.random((R, K, V, A)) < 0.4] = 0
    nv = rng.integers(0, V + 1, size=(R, K))
    for s in range(V):
        vclk[:, :, s][nv <= s] = 0
    vval = rng.integers(0, 7, size=(R, K, V)).astype(np.uint64)
    D = int(rng.integers(0, R // 2 + 2)) if D is None else D
    def_row = np.sort(rng.integers(0, R, size=D)).astype(np.uint64)
    def_clock = rng.integers(0, cmax + 2, size=(D, A)).astype(np.uint64)
    Kw = (K + 63) // 64
    def_keys = np.zeros((D, Kw), np.uint64)
    for d in range(D):
        n = int(rng.integers(1, K + 1)) if keys_per_rm is None else min(K, keys_per_rm)
        for k in rng.choice(K, size=n, replace=False):
            def_keys[d, k // 64] |= np.uint64(1) << np.uint64(k % 64)
    return dict(clock=clock, ec=ec, vclk=vclk, vval=vval, def_row=def_row, def_clock=def_clock,
                def_keys=def_keys)


@pytest.mark.parametrize("seed,R,K,A,V,cmax", [
    (1, 1, 1, 1, 1, 4), (2, 7, 3, 2, 2, 5), (3, 40, 9, 4, 2, 6), (4, 25, 5, 33, 2, 3),
    (5, 12, 4, 64, 1, 3), (6, 10, 6, 65, 1, 3), (7, 6, 3, 200, 1, 3), (8, 50, 130, 3, 3, 5),
    (9, 30, 8, 8, 2, 4), (10, 33, 2, 5, 2, 1000), (11, 16, 5, 100, 2, 2), (12, 64, 3, 2, 4, 3),
])
def test_map_lub_many_arbitrary(mctx, seed, R, K, A, V, cmax):
    """Arbitrary dense states: exactness of the left fold does not rest on any invariant."""
    rng = np.random.default_rng(seed)
    d = _random_dense(rng, R, K, A, V, cmax)
    peak = np.zeros(K, np.uint64)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                     d["def_keys"], 64, peak=peak)
    vout = max(1, int(exp[4].max()) if exp[4].size else 1)
    if int(peak.max()) > 16:  # beyond the kernel's state capacity: must be reported, not wrong
        with pytest.raises(cg.map.MapCapacityError):
            _gpu(mctx, d, vout)
        return
    _check(mctx, d, vout)


def test_map_many_concurrent_deferred(mctx):
    """More than the 4 register-tracked removes active on one key: the rescan path."""
    rng = np.random.default_rng(77)
    R, K, A = 40, 3, 4
    d = _random_dense(rng, R, K, A, 2, cmax=3, D=60, keys_per_rm=K)
    d["def_clock"][:, 0] = 50  # never dominated: every remove stays active to the end
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                     d["def_keys"], 64)
    _check(mctx, d, max(1, int(exp[4].max())))


def test_map_groups(mctx):
    G, R, K, A = 3, 15, 10, 5
    parts = []
    for g in range(G):
        maps = O.gen_map_replicas(500 + g, R, K, A, steps=150, p_rm=0.3, p_up=0.4)
        parts.append(O.map_to_dense(maps, K, A, 3))
    st = {k: np.stack([p[k] for p in parts]) for k in ("clock", "ec", "vclk", "vval")}
    st["def_row"] = np.concatenate([p["def_row"] for p in parts])
    st["def_clock"] = np.concatenate([p["def_clock"] for p in parts])
    st["def_keys"] = np.concatenate([p["def_keys"] for p in parts])
    counts = [p["def_row"].shape[0] for p in parts]
    res, kw = _gpu(mctx, st, 6, groups=counts)
    off = np.cumsum([0] + counts)
    for g, p in enumerate(parts):
        exp = O.map_fold(p["clock"], p["ec"], p["vclk"], p["vval"], p["def_row"], p["def_clock"],
                         p["def_keys"], 6)
        np.testing.assert_array_equal(to_host(res.clock[g]), exp[0])
        np.testing.assert_array_equal(to_host(res.ec[g]), exp[1])
        np.testing.assert_array_equal(to_host(res.vclk[g]), exp[2])
        np.testing.assert_array_equal(to_host(res.vval[g]), exp[3])
        got = cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys, int(off[g]), int(off[g + 1])) if kw else set()
        assert got == exp[5]


def test_map_empty_and_errors(gpu_ctx):
    A, K = 3, 4
    z = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    res = cg.map.lub_many(z(0, A), z(0, K, A), z(0, K, 2, A), z(0, K, 2), ctx=gpu_ctx)
    assert not to_host(res.clock).any() and not to_host(res.ec).any() and not to_host(res.vclk).any()
    # capacity: three concurrent values folded into vout=2 slots
    rng = np.random.default_rng(3)
    clock = np.zeros((3, A), np.uint64)
    ec = np.zeros((3, K, A), np.uint64)
    vclk = np.zeros((3, K, 1, A), np.uint64)
    vval = np.zeros((3, K, 1), np.uint64)
    for r in range(3):
        clock[r, r] = ec[r, 0, r] = vclk[r, 0, 0, r] = 1
        vval[r, 0, 0] = 10 + r
    with pytest.raises(cg.map.MapCapacityError):
        cg.map.lub_many(to_dev(clock), to_dev(ec), to_dev(vclk), to_dev(vval), vout=2, ctx=gpu_ctx)
    res = cg.map.lub_many(to_dev(clock), to_dev(ec), to_dev(vclk), to_dev(vval), vout=3, ctx=gpu_ctx)
    assert res.nval.cpu().tolist()[0] == 3
    assert to_host(res.vval)[0].tolist() == [10, 11, 12]
    # unsorted deferred rows are reported
    d = _random_dense(rng, 6, K, A, 1, 4, D=3)
    d["def_row"] = np.array([4, 1, 2], np.uint64)
    with pytest.raises(ValueError):
        _gpu(gpu_ctx, d, 8)


def test_synth_map_matches_cpu(gpu_ctx):
    from crdts_gpu import synth
    seed, R, K, A, V, kmax = 11, 90, 70, 9, 3, 30
    inp = synth.map_replicas(gpu_ctx, R, K, A, V, seed, kmax=kmax, p_def=0.3)
    dfr = O.synth_map_deferred(seed, R, K, A, kmax, p_def=0.3)
    exp = O.synth_map(seed, R, K, A, V, kmax, deferred=dfr)
    for nm in ("clock", "ec", "vclk", "vval"):
        np.testing.assert_array_equal(to_host(getattr(inp, nm)), exp[nm], err_msg=nm)
    assert inp.def_clock.shape[0] == len(dfr[0]) > 0
    np.testing.assert_array_equal(to_host(inp.def_clock), dfr[1])
    np.testing.assert_array_equal(to_host(inp.def_keys), dfr[2])


@pytest.mark.parametrize("R,K,A,kmax", [(4096, 256, 32, 64), (3000, 100, 7, 40), (2000, 64, 64, 30), (1500, 40, 2, 9)])
def test_map_synth_sampled_keys(mctx, R, K, A, kmax):
    """Synthetic replicas in HBM, folded on the GPU; the oracle folds a key sample over every
    replica (keys are independent given the clocks) and must match bit for bit."""
    from crdts_gpu import synth
    seed = 0x5EED0004
    inp = synth.map_replicas(mctx, R, K, A, 2, seed, kmax=kmax, p_def=0.1)
    res = cg.map.lub_many(inp.clock, inp.ec, inp.vclk, inp.vval, def_off=inp.def_off,
                          def_row=inp.def_row, def_clock=inp.def_clock, def_keys=inp.def_keys,
                          vout=4, ctx=mctx)
    keys = np.random.default_rng(R).choice(K, size=8, replace=False)
    dfr = O.synth_map_deferred(seed, R, K, A, kmax, p_def=0.1)
    d = O.synth_map(seed, R, K, A, 2, kmax, keys=keys, deferred=dfr)
    sub_keys = O.restrict_deferred_keys(dfr[2], keys)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], dfr[0], dfr[1], sub_keys, 4)
    np.testing.assert_array_equal(to_host(res.clock), exp[0])
    np.testing.assert_array_equal(to_host(res.ec)[keys], exp[1])
    np.testing.assert_array_equal(to_host(res.vclk)[keys], exp[2])
    np.testing.assert_array_equal(to_host(res.vval)[keys], exp[3])
    np.testing.assert_array_equal(res.nval.cpu().numpy()[keys], exp[4])
    # surviving deferred removes restricted to the sample
    got = cg.map.deferred_set(inp.def_clock, res.def_keep, res.def_keys)
    pos = {int(k): i for i, k in enumerate(keys)}
    got_sub = set()
    for c, ks in got:
        sub = frozenset(pos[k] for k in ks if k in pos)
        if sub:
            got_sub.add((c, sub))
    exp_sub = {(c, ks) for c, ks in exp[5] if ks}
    assert got_sub == exp_sub


def _chain_dense(rng, R, K, A, V, cmax, nchain=3):
    """_random_dense with single-actor value clocks drawn from nchain actors per key, distinct
    within a replica's register: every fold state then holds at most nchain values per key
    (values on one actor are totally ordered), so wide-A shapes fit the 4-slot LDS-DMA path."""
    d = _random_dense(rng, R, K, A, V, cmax, D=(0 if R == 1 else max(1, R // 3)), keys_per_rm=max(1, K // 4))
    sparse = rng.random(d["def_clock"].shape) < 2.0 / A  # removes name ~2 actors: some keys survive
    d["def_clock"] = np.where(sparse, d["def_clock"], 0).astype(np.uint64)
    chains = np.stack([rng.choice(A, size=min(nchain, A), replace=False) for _ in range(K)])
    vclk = np.zeros_like(d["vclk"])
    for r in range(R):
        for k in range(K):
            acts = rng.permutation(chains[k])
            for s in range(V):
                if d["vclk"][r, k, s].any() and s < acts.shape[0]:
                    vclk[r, k, s, acts[s]] = rng.integers(1, cmax + 1)
    d["vclk"] = vclk
    return d


@pytest.mark.parametrize("seed,R,K,A,V", [(21, 37, 9, 2, 1), (22, 70, 5, 8, 2), (23, 19, 6, 64, 2),
                                         (24, 50, 12, 32, 2), (25, 33, 3, 16, 1), (26, 1, 4, 4, 2),
                                         (27, 200, 40, 32, 2), (28, 45, 7, 64, 1)])
def test_map_even_actor_shapes(mctx, seed, R, K, A, V):
    """Shapes the LDS-DMA staging takes (A even, V <= 2, 4 output slots), incl. partial chunks and
    config 4's own A = 32, V = 2.  Value clocks are per-key actor chains so that no fold needs
    more than 4 values: every case runs (none is skipped)."""
    rng = np.random.default_rng(seed)
    d = _chain_dense(rng, R, K, A, V, cmax=6)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                     d["def_keys"], 64)
    assert int(exp[4].max() if exp[4].size else 0) <= 4
    assert d["def_row"].shape[0] > 0 or R == 1
    assert exp[4].any()  # some register survives the fold
    _check(mctx, d, 4)


def test_map_direct_remove_walk(mctx):
    """More removes naming one key than the per-key LDS list holds (kMapL = 256): the fold walks
    the group's remove list directly, with even A and V <= 2, so the RS and LDS-DMA paths take it."""
    rng = np.random.default_rng(91)
    R, K, A = 700, 2, 4
    d = _chain_dense(rng, R, K, A, 2, cmax=8)
    D = 300
    d["def_row"] = np.sort(rng.integers(0, R, size=D)).astype(np.uint64)
    d["def_clock"] = np.where(rng.random((D, A)) < 0.5, rng.integers(1, 9, size=(D, A)), 0).astype(np.uint64)
    d["def_keys"] = np.full((D, 1), 3, np.uint64)  # both keys
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                     d["def_keys"], 64)
    assert int(exp[4].max() if exp[4].size else 0) <= 4
    _check(mctx, d, 4)


@pytest.mark.parametrize("seed,R,A", [(31, 1000, 32), (32, 517, 16), (33, 263, 8)])
def test_map_long_folds_mixed_chunks(mctx, seed, R, A):
    """Long folds (many 16-replica chunks, a partial last one) where most chunks are skipped whole
    and a few carry removes or changes: the RS path's hand-over to the exact loop and back."""
    rng = np.random.default_rng(seed)
    d = _chain_dense(rng, R, 6, A, 2, cmax=40)
    # mostly old replicas: clocks and entries well below the running max, so most steps are no-ops
    old = rng.random(R) < 0.9
    d["ec"][old] = np.minimum(d["ec"][old], 2).astype(np.uint64)
    d["vclk"][old] = np.minimum(d["vclk"][old], 2).astype(np.uint64)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                     d["def_keys"], 64)
    if int(exp[4].max() if exp[4].size else 0) > 4:
        pytest.skip("fold needs more than 4 values")
    _check(mctx, d, 4)


@pytest.mark.parametrize("R,V", [(12, 1), (2, 6), (2, 8), (3, 6), (1, 7)])
def test_map_many_concurrent_values(mctx, R, V):
    """Registers with many concurrent values: inputs with up to 8 values per key (V > 4) and folds
    whose state needs 9-16 values (the 16-value state, exact steps only); 18 concurrent values
    exceed the state and are reported."""
    K, A = 3, 24
    clock = np.zeros((R, A), np.uint64)
    ec = np.zeros((R, K, A), np.uint64)
    vclk = np.zeros((R, K, V, A), np.uint64)
    vval = np.zeros((R, K, V), np.uint64)
    for r in range(R):
        for t in range(V):  # replica r holds V concurrent writes, every write by its own actor
            a = r * V + t
            clock[r, a] = 1
            ec[r, :, a] = 1
            vclk[r, :, t, a] = 1
            vval[r, :, t] = 100 * r + t
    d = dict(clock=clock, ec=ec, vclk=vclk, vval=vval, def_row=np.zeros(0, np.uint64),
             def_clock=np.zeros((0, A), np.uint64), def_keys=np.zeros((0, 1), np.uint64))
    peak = np.zeros(K, np.uint64)
    exp = O.map_fold(clock, ec, vclk, vval, d["def_row"], d["def_clock"], d["def_keys"], 64, peak=peak)
    assert int(exp[4].max()) == R * V
    if R * V > 16:
        with pytest.raises(cg.map.MapCapacityError):
            _gpu(mctx, d, R * V)
        return
    _check(mctx, d, R * V)


def _old_heavy(rng, R, K, A, G=1, D=None):
    """_chain_dense at A = 32, V = 2 with mostly old replicas (most chunks skipped whole, a few
    handed to the exact loop), stacked over G groups."""
    parts = []
    for _ in range(G):
        d = _chain_dense(rng, R, K, A, 2, cmax=40)
        old = rng.random(R) < 0.9
        d["ec"][old] = np.minimum(d["ec"][old], 2).astype(np.uint64)
        d["vclk"][old] = np.minimum(d["vclk"][old], 2).astype(np.uint64)
        parts.append(d)
    return parts


@pytest.mark.parametrize("R", [1, 3, 15, 16, 17, 31, 32, 33, 48, 63, 64, 65, 80, 81, 97, 113, 150, 1000])
def test_map_shared_ring_chunk_counts(mctx, R):
    """The SH path (msh=1: four key waves per workgroup sharing each chunk's clock rows through a ring of
    shared LDS slots) at every chunk count around its prologue / ring depth (1..9 chunks and past
    it), partial last chunks, K = 8 keys (two workgroups); results must equal the oracle fold in
    every staging mode."""
    rng = np.random.default_rng(4000 + R)
    d = _old_heavy(rng, R, 8, 32)[0]
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                     d["def_keys"], 64)
    if int(exp[4].max() if exp[4].size else 0) > 4:
        pytest.skip("fold needs more than 4 values")
    _check(mctx, d, 4)


@pytest.mark.parametrize("seed,R,K", [(41, 300, 4), (42, 777, 12), (43, 64, 16)])
def test_map_shared_ring_groups(mctx, seed, R, K):
    """SH path over several groups (each workgroup's four keys inside one group, groups with their
    own clock rows and deferred lists)."""
    rng = np.random.default_rng(seed)
    G = 3
    parts = _old_heavy(rng, R, K, 32, G=G)
    st = {k: np.stack([p[k] for p in parts]) for k in ("clock", "ec", "vclk", "vval")}
    st["def_row"] = np.concatenate([p["def_row"] for p in parts])
    st["def_clock"] = np.concatenate([p["def_clock"] for p in parts])
    st["def_keys"] = np.concatenate([p["def_keys"] for p in parts])
    counts = [p["def_row"].shape[0] for p in parts]
    exps = [O.map_fold(p["clock"], p["ec"], p["vclk"], p["vval"], p["def_row"], p["def_clock"], p["def_keys"], 64)
            for p in parts]
    if max(int(e[4].max() if e[4].size else 0) for e in exps) > 4:
        pytest.skip("fold needs more than 4 values")
    exps = [O.map_fold(p["clock"], p["ec"], p["vclk"], p["vval"], p["def_row"], p["def_clock"], p["def_keys"], 4)
            for p in parts]
    res, kw = _gpu(mctx, st, 4, groups=counts)
    off = np.cumsum([0] + counts)
    for g, exp in enumerate(exps):
        np.testing.assert_array_equal(to_host(res.clock[g]), exp[0])
        np.testing.assert_array_equal(to_host(res.ec[g]), exp[1])
        np.testing.assert_array_equal(to_host(res.vclk[g]), exp[2])
        np.testing.assert_array_equal(to_host(res.vval[g]), exp[3])
        np.testing.assert_array_equal(res.nval[g].cpu().numpy(), exp[4])
        got = cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys, int(off[g]), int(off[g + 1])) if kw else set()
        assert got == exp[5]
