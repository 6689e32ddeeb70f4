"""GPU parity of the causal helpers (crdt_vclock_pair_op / partial_cmp / cmp_matrix,
crdt_gcounter_read / crdt_pncounter_read) against the oracle's restatement of vclock.rs:68-80,
:95-105, :246-259, gcounter.rs:70-72 and pncounter.rs:110-115 (VClock objects, Python ints).
The reference's own KATs for these ops run on the GPU in test_gpu_kat.py::test_kat_gpu_causal."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402

CODE = {O.EQUAL: 0, O.GREATER: 1, O.LESS: -1, O.NONE: 2}


def _vc(row):
    return O.VClock({a: int(c) for a, c in enumerate(row) if c})


def _dense(vc, A):
    r = np.zeros(A, np.uint64)
    for a, c in vc.dots.items():
        r[a] = c
    return r


def _pairs(rng, N, A, cmax):
    """Row pairs covering every ordering: equal, dominated either way, concurrent."""
    x = rng.integers(0, cmax, size=(N, A)).astype(np.uint64)
    x[rng.random((N, A)) < 0.3] = 0
    y = x.copy()
    kind = rng.integers(0, 4, size=N)
    for i in range(N):
        if kind[i] == 1:
            y[i] = np.minimum(x[i], rng.integers(0, cmax, size=A).astype(np.uint64))
        elif kind[i] == 2:
            y[i] = np.maximum(x[i], rng.integers(0, cmax, size=A).astype(np.uint64))
        elif kind[i] == 3:
            y[i] = rng.integers(0, cmax, size=A).astype(np.uint64)
    return x, y


@pytest.mark.parametrize("N,A,cmax", [(500, 64, 5), (333, 7, 4), (64, 300, 1 << 63), (1, 1, 3), (257, 130, 9)])
def test_glb_forget_cmp(gpu_ctx, N, A, cmax):
    rng = np.random.default_rng(N + A)
    x, y = _pairs(rng, N, A, cmax)
    dx, dy = to_dev(x), to_dev(y)
    glb, fgt = to_host(cg.causal.glb(dx, dy)), to_host(cg.causal.forget(dx, dy))
    inter = to_host(cg.causal.intersection(dx, dy))
    cmpv = cg.causal.partial_cmp(dx, dy).cpu().numpy()
    conc = cg.causal.concurrent(dx, dy).cpu().numpy()
    for i in range(N):
        a, b = _vc(x[i]), _vc(y[i])
        g = a.copy()
        g.glb(b)
        f = a.copy()
        f.forget(b)
        assert np.array_equal(glb[i], _dense(g, A)), i
        assert np.array_equal(fgt[i], _dense(f, A)), i
        assert np.array_equal(inter[i], _dense(O.VClock.intersection(a, b), A)), i
        assert cmpv[i] == CODE[a.partial_cmp(b)], i
        assert bool(conc[i]) == (a.partial_cmp(b) is O.NONE), i
    assert set(cmpv.tolist()) >= ({0, 1, -1, 2} if N > 100 else set())


def test_pair_ops_in_place_and_strided(gpu_ctx):
    rng = np.random.default_rng(5)
    x, y = _pairs(rng, 200, 40, 6)
    big = to_dev(np.concatenate([x, y, y], axis=1))  # rows of 120 words, x at 0, y at 40
    dx, dy = big[:, :40], big[:, 40:80]
    exp = [_vc(x[i]) for i in range(200)]
    for i, e in enumerate(exp):
        e.forget(_vc(y[i]))
    cg.causal.forget(dx, dy, out=dx)  # in place, strided rows
    got = to_host(big)[:, :40]
    assert all(np.array_equal(got[i], _dense(exp[i], 40)) for i in range(200))


@pytest.mark.parametrize("N,A", [(300, 70), (64, 1), (129, 33)])
def test_cmp_matrix(gpu_ctx, N, A):
    rng = np.random.default_rng(N)
    base = rng.integers(0, 4, size=(N, A)).astype(np.uint64)
    base[::7] = base[0]  # some equal clocks
    m = cg.causal.cmp_matrix(to_dev(base)).cpu().numpy()
    # dense restatement of partial_cmp over all pairs, itself checked against the oracle on a sample
    ge = (base[:, None, :] >= base[None, :, :]).all(-1)
    le = (base[:, None, :] <= base[None, :, :]).all(-1)
    exp = np.where(ge & le, 0, np.where(ge, 1, np.where(le, -1, 2))).astype(np.int8)
    for i, j in zip(rng.integers(0, N, 500), rng.integers(0, N, 500)):
        assert exp[i, j] == CODE[_vc(base[i]).partial_cmp(_vc(base[j]))]
    np.testing.assert_array_equal(m, exp)


@pytest.mark.parametrize("N,A,full", [(400, 256, False), (50, 1000, True), (3, 1, True)])
def test_counter_read(gpu_ctx, N, A, full):
    """Exact sums; full-range u64 counters carry past 2^64 (no KAT covers that range:
    parity there is against the oracle's unbounded Python-int restatement only)."""
    rng = np.random.default_rng(A)
    hi = (1 << 64) - 1 if full else 1000
    g = rng.integers(0, hi, size=(N, A), dtype=np.uint64, endpoint=True)
    got = cg.gcounter.read(to_dev(g))
    for i in range(N):
        c = O.GCounter()
        c.inner = _vc(g[i])
        assert got[i] == c.read()
    pn = rng.integers(0, hi, size=(N, 2 * A), dtype=np.uint64, endpoint=True)
    got = cg.pncounter.read(to_dev(pn))
    for i in range(N):
        c = O.PNCounter()
        c.p.inner, c.n.inner = _vc(pn[i, :A]), _vc(pn[i, A:])
        assert got[i] == c.read()
    assert cg.gcounter.read(to_dev(g[0])) == got_single(g[0])


def got_single(row):
    return sum(int(x) for x in row)


def test_vclock_module_api(gpu_ctx):
    """crdts_gpu.vclock mirrors src/vclock.rs's batch-able surface: each call against the oracle's
    VClock methods on the same rows (vclock.rs:68-80, :95-105, :125-159, :148-152, :201-259)."""
    rng = np.random.default_rng(21)
    x, y = _pairs(rng, 300, 24, 6)
    dx, dy = to_dev(x), to_dev(y)
    vc = cg.vclock
    out = {"glb": to_host(vc.glb(dx, dy)), "forget": to_host(vc.forget(dx, dy)),
           "clone_without": to_host(vc.clone_without(dx, dy)), "intersection": to_host(vc.intersection(dx, dy)),
           "merge": to_host(vc.merge_batch(dx.clone(), dy))}
    cmpv, conc = vc.partial_cmp(dx, dy).cpu().numpy(), vc.concurrent(dx, dy).cpu().numpy()
    for i in range(300):
        a, b = _vc(x[i]), _vc(y[i])
        g = a.copy()
        g.glb(b)
        m = a.copy()
        m.merge(b)
        assert np.array_equal(out["glb"][i], _dense(g, 24))
        assert np.array_equal(out["forget"][i], _dense(a.clone_without(b), 24))
        assert np.array_equal(out["clone_without"][i], _dense(a.clone_without(b), 24))
        assert np.array_equal(out["intersection"][i], _dense(O.VClock.intersection(a, b), 24))
        assert np.array_equal(out["merge"][i], _dense(m, 24))
        assert cmpv[i] == CODE[a.partial_cmp(b)] and bool(conc[i]) == a.concurrent(b)
    assert np.array_equal(to_host(dx), x)  # forget / glb / intersection without out= leave x alone
    # CmRDT::apply of Dot ops in stream order, and the fold
    st = to_dev(x[:50].copy())
    n = 2000
    idx, act = rng.integers(0, 50, n), rng.integers(0, 24, n)
    ctr = rng.integers(0, 9, n).astype(np.uint64)
    assert vc.apply(st, torch.from_numpy(idx.astype(np.int32)).cuda(), torch.from_numpy(act.astype(np.int32)).cuda(),
                    to_dev(ctr)) == 0
    exp = [_vc(x[i]) for i in range(50)]
    for i, a, c in zip(idx, act, ctr):
        exp[i].apply(O.Dot(int(a), int(c)))
    assert all(np.array_equal(to_host(st)[i], _dense(exp[i], 24)) for i in range(50))
    acc = O.VClock()
    for i in range(300):
        acc.merge(_vc(x[i]))
    assert np.array_equal(to_host(vc.lub_many(dx)), _dense(acc, 24))
    assert np.array_equal(vc.cmp_matrix(dx[:40]).cpu().numpy(), cg.causal.cmp_matrix(dx[:40]).cpu().numpy())


def test_gset_module_api(gpu_ctx):
    """crdts_gpu.gset: insert ops (gset.rs:46-48, :69-71), contains (:83-85), read (:103-105) and
    the fold (:38-40) against the oracle's GSet on the same interned elements."""
    rng = np.random.default_rng(22)
    N, U = 40, 200
    W = (U + 63) // 64
    st = torch.zeros((N, W), dtype=torch.int64, device="cuda")
    n = 3000
    idx, el = rng.integers(0, N, n), rng.integers(0, U, n)
    assert cg.gset.apply(st, torch.from_numpy(idx.astype(np.int32)).cuda(),
                         torch.from_numpy(el.astype(np.int32)).cuda(), U) == 0
    exp = [O.GSet() for _ in range(N)]
    for i, e in zip(idx, el):
        exp[i].insert(int(e))
    vals = torch.arange(U, dtype=torch.int64) * 7 + 3  # interning dictionary: position -> value
    assert cg.gset.read(st) == [sorted(e.value) for e in exp]
    assert cg.gset.read(st, vals) == [[7 * p + 3 for p in sorted(e.value)] for e in exp]
    probe = torch.from_numpy(rng.integers(-5, U + 70, N)).cuda()
    got = cg.gset.contains(st, probe).cpu().numpy()
    assert [bool(g) for g in got] == [exp[i].contains(int(p)) for i, p in enumerate(probe.tolist())]
    acc = O.GSet()
    for e in exp:
        acc.merge(e)
    assert cg.gset.read(cg.gset.lub_many(st).unsqueeze(0)) == [sorted(acc.value)]


def test_device_empty_block(gpu_ctx):
    """crdt_device_alloc (one physically contiguous block) seen as a torch tensor: the fold reads it
    like any other replica batch, and the block is freed with its last view."""
    t = gpu_ctx.device_empty((1000, 64))
    assert t is not None and t.shape == (1000, 64) and t.dtype == torch.int64 and t.device.index == gpu_ctx.device
    rng = np.random.default_rng(9)
    x = rng.integers(0, 1 << 40, size=(1000, 64)).astype(np.uint64)
    t.copy_(to_dev(x))
    assert np.array_equal(to_host(cg.vclock.lub_many(t, ctx=gpu_ctx)), x.max(axis=0))
    v = t[10:20]
    del t
    assert np.array_equal(to_host(v), x[10:20])  # the view keeps the block alive
    del v
    assert gpu_ctx.device_empty((0,)) is not None
