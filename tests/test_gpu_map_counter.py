"""GPU parity: Map<K, GCounter> / Map<K, PNCounter> lub_many (crdt_map_counter_lub_many, round 4)
against the oracle's left fold of Map::merge (map.rs:140-220) with the counter's merge / forget
(gcounter.rs:44-54, pncounter.rs:70-82).  The fold is not associative for these values (checked in
tests/test_oracle_map_counter.py), so the kernel folds each key in replica order; these cases
cover op-replay replicas (writes, removes, out-of-order delivery that leaves deferred removes),
arbitrary dense states, groups, wide actor sets (A = 100, 300), many live removes on one key, an
empty fold and unsorted def_row."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


@pytest.fixture(params=["mckpw=0", "mckpw=1", "mckpw=2", "mckpw=4", "mcdma=8", "mcdma=16", "mccs=0", "mccl=1"])
def mcctx(request):
    """The default (A = 32 / 16 / 8: the whole-chunk skip with register-staged chunks, round 5; otherwise
    the register ring with keys per wave chosen by the grid size), 1, up to 2 or up to 4 keys per
    wave (A <= 64 / keys), the replica rows by LDS-DMA into an 8- or 16-slot LDS ring (A even,
    (2+W)*A <= 128; one key per wave), the register ring without the chunk skip (mccs=0), or the
    chunk skip with LDS-staged chunks (mccl=1, opt-in).  Shapes outside a mode's bound take the one-key
    register ring."""
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    ctx.tune(request.param)
    yield ctx
    ctx.close()


def _run(ctx, d, G=1, off=None, check=True):
    """d: dense replicas (clock (R,A), ec (R,K,A), val (R,K,W,A), def_row/def_clock/def_keys) of one
    group, or G groups stacked when off (per-group CSR offsets of the pool) is given."""
    R = d["clock"].shape[0] // G
    shp = lambda x: x.reshape((G, R) + x.shape[1:])  # noqa: E731
    D = d["def_row"].shape[0]
    kw = {}
    if D:
        kw = dict(def_off=off if off is not None else [0, D],
                  def_row=torch.from_numpy(np.asarray(d["def_row"], np.int64).astype(np.int32)).cuda(),
                  def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"]))
    return cg.map.counter_lub_many(to_dev(shp(d["clock"])), to_dev(shp(d["ec"])), to_dev(shp(d["val"])), ctx=ctx,
                                   check=check, **kw), kw


def _got_maps(res, kw, G):
    out = []
    c, e, v = to_host(res.clock), to_host(res.ec), to_host(res.val)
    for g in range(G):
        dset = set()
        if kw:
            off = kw["def_off"]
            dset = cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys, int(off[g]), int(off[g + 1]))
        out.append(O.dense_to_map_counter(c[g], e[g], v[g], [(np.array(rm, np.uint64), ks) for rm, ks in dset]))
    return out


def _same(got, exp):
    assert got.clock == exp.clock
    assert got.entries == exp.entries
    assert got.deferred == exp.deferred


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("seed,R,K,A", [(1, 40, 6, 5), (2, 60, 12, 8), (3, 25, 3, 4), (4, 90, 20, 12)])
def test_map_counter_op_replay(mcctx, W, seed, R, K, A):
    maps = O.map_counter_objects(R, K, A, W, seed=seed, steps=6 * R, p_rm=0.3)
    exp = O.map_fold_objects(maps)
    d = O.map_counter_to_dense(maps, K, A, W)
    res, kw = _run(mcctx, d)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


def _arbitrary(rng, R, K, A, W, cmax, ndef):
    """Random dense states (no well-formedness), each replica's deferred removes with random key sets."""
    maps = []
    for _ in range(R):
        clock = rng.integers(0, cmax + 1, size=A).astype(np.uint64)
        ec = rng.integers(0, cmax + 2, size=(K, A)).astype(np.uint64) * (rng.random((K, A)) < 0.4)
        val = rng.integers(0, cmax + 3, size=(K, W, A)).astype(np.uint64) * (rng.random((K, W, A)) < 0.5)
        deferred = []
        for _ in range(int(rng.integers(0, ndef + 1))):
            rm = rng.integers(0, cmax + 3, size=A).astype(np.uint64) * (rng.random(A) < 0.4)
            if rm.any() and not any(np.array_equal(rm, x) for x, _ in deferred):
                deferred.append((rm, set(int(k) for k in rng.choice(K, size=int(rng.integers(1, K + 1)),
                                                                     replace=False))))
        maps.append(O.dense_to_map_counter(clock, ec.astype(np.uint64), val.astype(np.uint64), deferred))
    return maps


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("seed,R,K,A,cmax", [(11, 30, 5, 6, 4), (12, 50, 3, 3, 3), (13, 20, 9, 64, 5),
                                             (14, 16, 4, 100, 3), (15, 12, 3, 300, 4)])
def test_map_counter_arbitrary(mcctx, W, seed, R, K, A, cmax):
    rng = np.random.default_rng(seed)
    maps = _arbitrary(rng, R, K, A, W, cmax, 2)
    exp = O.map_fold_objects(maps)
    d = O.map_counter_to_dense(maps, K, A, W)
    res, kw = _run(mcctx, d)
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.mark.parametrize("W", [1, 2])
def test_map_counter_groups(mcctx, W):
    """G = 4 groups of one launch, each with its own slice of the pooled removes (CSR offsets)."""
    G, R, K, A = 4, 30, 7, 6
    parts = [O.map_counter_objects(R, K, A, W, seed=40 + g, steps=200, p_rm=0.35) for g in range(G)]
    ds = [O.map_counter_to_dense(p, K, A, W) for p in parts]
    cat = {k: np.concatenate([x[k] for x in ds]) for k in ("clock", "ec", "val", "def_clock", "def_keys")}
    cat["def_row"] = np.concatenate([x["def_row"] for x in ds])
    off = np.cumsum([0] + [x["def_row"].shape[0] for x in ds]).tolist()
    assert off[-1] > 0
    res, kw = _run(mcctx, cat, G=G, off=off)
    got = _got_maps(res, kw, G)
    for g in range(G):
        _same(got[g], O.map_fold_objects(parts[g]))


def test_map_counter_many_live_removes(mcctx):
    """40 removes naming key 0 stay deferred (future clocks on an actor no replica reaches): more
    than the LDS row cache holds, so the rest are re-read from HBM every step; all survive."""
    R, K, A, W = 24, 2, 4, 1
    rng = np.random.default_rng(7)
    maps = []
    for r in range(R):
        m = O.Map(O.GCounter)
        m.clock = O.VClock({0: r + 1})
        g = O.GCounter()
        g.inner = O.VClock({0: r + 1, 1: int(rng.integers(1, 5))})
        m.entries[0] = O.MapEntry(O.VClock({0: r + 1}), g)
        if r < 20:
            for t in range(2):
                m.deferred[O.VClock({0: int(rng.integers(1, 30)), 3: 100 + 2 * r + t})] = {0}
        maps.append(m)
    exp = O.map_fold_objects(maps)
    assert len(exp.deferred) == 40
    d = O.map_counter_to_dense(maps, K, A, W)
    res, kw = _run(mcctx, d)
    _same(_got_maps(res, kw, 1)[0], exp)


def test_map_counter_empty_and_unsorted(gpu_ctx):
    """R = 0 folds to Map::new(); a def_row that decreases is flagged (bit 1), not silently used."""
    z = torch.zeros((2, 0, 4), dtype=torch.int64, device="cuda:0")
    res = cg.map.counter_lub_many(z, torch.zeros((2, 0, 3, 4), dtype=torch.int64, device="cuda:0"),
                                  torch.zeros((2, 0, 3, 1, 4), dtype=torch.int64, device="cuda:0"), ctx=gpu_ctx)
    assert not to_host(res.clock).any() and not to_host(res.ec).any() and not to_host(res.val).any()
    maps = O.map_counter_objects(20, 4, 4, 1, seed=9, steps=200, p_rm=0.4)
    d = O.map_counter_to_dense(maps, 4, 4, 1)
    if d["def_row"].shape[0] < 2:
        pytest.skip("needs two removes")
    d["def_row"] = d["def_row"][::-1].copy()
    if (np.diff(d["def_row"].astype(np.int64)) >= 0).all():
        pytest.skip("reversal did not unsort")
    with pytest.raises(ValueError, match="def_row"):
        _run(gpu_ctx, d)


@pytest.mark.parametrize("W", [1, 2])
def test_map_counter_remove_empties_last_actor(mcctx, W):
    """A deferred remove empties an entry whose only dot is on the last actor (A = 5: lanes past A
    hold copies of actor A-1, remove rows included), leaving a stale value behind; the next
    replica re-adds the key, which must read as absent-then-added (value v2 forgotten by
    we_deleted), not as a join with the stale value."""
    A = 5

    def cnt(dots):
        g = O.GCounter()
        g.inner = O.VClock(dots)
        if W == 1:
            return g
        c = O.PNCounter()
        c.p.inner = g.inner
        c.n.inner = O.VClock({a: x + 1 for a, x in dots.items()})
        return c

    r0 = O.Map(O.GCounter if W == 1 else O.PNCounter)
    r0.clock = O.VClock({4: 1})
    r0.entries[0] = O.MapEntry(O.VClock({4: 1}), cnt({3: 7}))
    r1 = O.Map(r0.vnew)
    r1.deferred[O.VClock({4: 1, 0: 5})] = {0}
    r2 = O.Map(r0.vnew)
    r2.clock = O.VClock({0: 1, 1: 1})
    r2.entries[0] = O.MapEntry(O.VClock({1: 1}), cnt({1: 3}))
    maps = [r0, r1, r2]
    exp = O.map_fold_objects(maps)
    assert exp.entries[0].val == cnt({1: 3})
    d = O.map_counter_to_dense(maps, 2, A, W)
    res, kw = _run(mcctx, d)
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.mark.parametrize("W", [1, 2])
def test_map_counter_auto_keys_per_wave_keeps_per_key_capacity(gpu_ctx, W):
    """with keys per wave chosen automatically (K = 4,096, A = 16: two keys per wave), keys 0
    and 1 share a wave and hold 300 live removes each (600 together, past the shared 512-entry list);
    the per-key limit of the header still holds — the group is re-folded one key per wave."""
    R, K, A = 4, 4096, 16
    vnew = O.GCounter if W == 1 else O.PNCounter
    maps = []
    for r in range(R):
        m = O.Map(vnew)
        m.clock = O.VClock({0: r + 1, 1: r + 1})
        for k in (0, 1, 2):
            v = vnew()
            (v.inner if W == 1 else v.p.inner).dots[k % A] = r + 2
            m.entries[k] = O.MapEntry(O.VClock({0: r + 1}), v)
        if r == 1:
            for i in range(300):
                m.deferred[O.VClock({3: 1000 + i})] = {0}
                m.deferred[O.VClock({5: 1000 + i})] = {1}
        maps.append(m)
    exp = O.map_fold_objects(maps)
    assert len(exp.deferred) == 600
    d = O.map_counter_to_dense(maps, K, A, W)
    res, kw = _run(gpu_ctx, d)  # the default ctx: mckpw=0 (automatic)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("A,seed", [(32, 21), (16, 22), (8, 23)])
def test_map_counter_chunk_skip_op_replay(mcctx, W, A, seed):
    """The whole-chunk skip's shapes (A = 32 / 16 / 8) over long op-replay folds: 16-replica chunks
    with and without removes naming the key, skipped and exact chunks, a partial last chunk."""
    R, K = 150, 6
    maps = O.map_counter_objects(R, K, A, W, seed=seed, steps=5 * R, p_rm=0.25)
    exp = O.map_fold_objects(maps)
    d = O.map_counter_to_dense(maps, K, A, W)
    res, kw = _run(mcctx, d)
    assert int(res.flags.cpu()[0]) == 0
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("A,R,cmax,seed", [(32, 64, 3, 31), (16, 80, 2, 32), (8, 96, 4, 33), (32, 48, 1, 34)])
def test_map_counter_chunk_skip_arbitrary(mcctx, W, A, R, cmax, seed):
    """Arbitrary dense states with small counters (equal words, zeros, stale values behind empty
    clocks) at the chunk-skip shapes: whatever the test decides, the result is the exact left fold."""
    rng = np.random.default_rng(seed)
    maps = _arbitrary(rng, R, 3, A, W, cmax, 1)
    exp = O.map_fold_objects(maps)
    d = O.map_counter_to_dense(maps, 3, A, W)
    res, kw = _run(mcctx, d)
    _same(_got_maps(res, kw, 1)[0], exp)


@pytest.mark.parametrize("W", [1, 2])
def test_map_counter_chunk_skip_steady_state(mcctx, W):
    """Replicas that repeat one key's state (every chunk after the first skippable), then a late
    change and a late remove: the skipped chunks only merge their clocks."""
    A, K, R = 32, 2, 200
    base = O.map_counter_objects(12, K, A, W, seed=41, steps=120, p_rm=0.0)
    fold = O.map_fold_objects(base)
    maps = [fold.copy() for _ in range(R)]
    for r in range(R):
        maps[r].clock = fold.clock.copy()
        maps[r].clock.apply(O.Dot(r % A, fold.clock.get(r % A) + 1 + r // A))  # clocks keep growing
    late = O.map_counter_objects(4, K, A, W, seed=42, steps=80, p_rm=0.4)
    maps[150] = late[-1]
    if late[-2].deferred:
        maps[170] = late[-2]
    exp = O.map_fold_objects(maps)
    d = O.map_counter_to_dense(maps, K, A, W)
    res, kw = _run(mcctx, d)
    _same(_got_maps(res, kw, 1)[0], exp)
