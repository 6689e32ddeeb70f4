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
    cmpv = cg.causal.partial_cmp(dx, dy).cpu().numpy()
    for i in range(N):
        a, b = _vc(x[i]), _vc(y[i])
        g = a.copy()
        g.glb(b)
        f = a.copy()
        f.forget(b)
        assert np.array_equal(glb[i], _dense(g, A)), i
        assert np.array_equal(fgt[i], _dense(f, A)), i
        assert cmpv[i] == CODE[a.partial_cmp(b)], i
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
