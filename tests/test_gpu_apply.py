"""GPU parity of batched CmRDT::apply (crdt_*_apply_batch) against the oracle applying the same
ops one by one (VClock::apply vclock.rs:125-127 / apply_dot :155-159, GCounter::apply
gcounter.rs:39-41, PNCounter::apply pncounter.rs:62-67, GSet::apply gset.rs:46-48), including
colliding ops on one cell, zero counters (no-ops) and out-of-range ops (skipped, counted)."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _i32(a):
    return torch.from_numpy(np.asarray(a, np.int64).astype(np.int32)).cuda()


def _vc(row):
    return O.VClock({a: int(c) for a, c in enumerate(row) if c})


@pytest.mark.parametrize("kind", ["vclock", "gcounter"])
@pytest.mark.parametrize("N,A,n_ops,cmax", [(100, 17, 5000, 50), (7, 3, 20000, 1 << 64), (1000, 256, 100000, 10)])
def test_apply_dots(gpu_ctx, kind, N, A, n_ops, cmax):
    rng = np.random.default_rng(N * A)
    init = rng.integers(0, min(cmax, 1 << 62), size=(N, A), dtype=np.uint64)
    init[rng.random((N, A)) < 0.5] = 0
    si = rng.integers(0, N, n_ops)
    ac = rng.integers(0, A, n_ops)
    ct = rng.integers(0, cmax, n_ops, dtype=np.uint64, endpoint=False) if cmax < (1 << 64) else \
        rng.integers(0, (1 << 64) - 1, n_ops, dtype=np.uint64, endpoint=True)
    st = to_dev(init)
    bad = cg.apply.apply_dots(kind, st, _i32(si), _i32(ac), to_dev(ct))
    assert bad == 0
    got = to_host(st)
    objs = [_vc(r) for r in init]
    for s, a, c in zip(si.tolist(), ac.tolist(), ct.tolist()):
        objs[s].apply(O.Dot(a, int(c)))
    for n in range(N):
        exp = np.zeros(A, np.uint64)
        for a, c in objs[n].dots.items():
            exp[a] = c
        assert np.array_equal(got[n], exp), n


def test_pncounter_apply(gpu_ctx):
    rng = np.random.default_rng(3)
    N, A, n_ops = 300, 12, 40000
    st = to_dev(np.zeros((N, 2 * A), np.uint64))
    si, ac = rng.integers(0, N, n_ops), rng.integers(0, A, n_ops)
    ct = rng.integers(1, 100, n_ops).astype(np.uint64)
    dr = rng.integers(0, 2, n_ops).astype(np.uint8)
    assert cg.apply.apply_dots("pncounter", st, _i32(si), _i32(ac), to_dev(ct),
                               dir=torch.from_numpy(dr).cuda()) == 0
    objs = [O.PNCounter() for _ in range(N)]
    for s, a, c, d in zip(si.tolist(), ac.tolist(), ct.tolist(), dr.tolist()):
        objs[s].apply((O.Dot(a, c), O.PNCounter.NEG if d else O.PNCounter.POS))
    got = to_host(st)
    for n in range(N):
        p = np.zeros(A, np.uint64)
        q = np.zeros(A, np.uint64)
        for a, c in objs[n].p.inner.dots.items():
            p[a] = c
        for a, c in objs[n].n.inner.dots.items():
            q[a] = c
        assert np.array_equal(got[n], np.concatenate([p, q]))
    assert cg.pncounter.read(st) == [o.read() for o in objs]


def test_gset_apply(gpu_ctx):
    rng = np.random.default_rng(4)
    N, U, n_ops = 200, 1000, 30000
    W = (U + 63) // 64
    st = to_dev(np.zeros((N, W), np.uint64))
    si, el = rng.integers(0, N, n_ops), rng.integers(0, U, n_ops)
    assert cg.apply.apply_inserts(st, _i32(si), _i32(el), U) == 0
    objs = [O.GSet() for _ in range(N)]
    for s, e in zip(si.tolist(), el.tolist()):
        objs[s].apply(e)
    got = to_host(st)
    for n in range(N):
        members = {w * 64 + b for w in range(W) for b in range(64) if (int(got[n, w]) >> b) & 1}
        assert members == objs[n].value


def test_apply_out_of_range_skipped(gpu_ctx):
    st = to_dev(np.zeros((4, 3), np.uint64))
    bad = cg.apply.apply_dots("vclock", st, _i32([0, 4, 1, 2]), _i32([1, 0, 3, 2]), to_dev(np.array([5, 6, 7, 8], np.uint64)))
    assert bad == 2
    exp = np.zeros((4, 3), np.uint64)
    exp[0, 1], exp[2, 2] = 5, 8
    assert np.array_equal(to_host(st), exp)
    g = to_dev(np.zeros((2, 1), np.uint64))
    assert cg.apply.apply_inserts(g, _i32([0, 1, 2]), _i32([63, 64, 0]), 64) == 2
