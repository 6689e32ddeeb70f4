"""GPU parity: LWWReg lub_many (state + exact first-conflict index) and merge_batch."""
import numpy as np
import pytest

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402

NONE = np.uint64(2**64 - 1)


def _inputs(seed, G, R, mod=None, vmod=None):
    m = O.synth_matrix(seed, G, R, 2)
    v = O.synth_matrix(seed, G, R, 3)
    if mod:
        m = m % np.uint64(mod)
    if vmod:
        v = v % np.uint64(vmod)
    return m, v


@pytest.mark.parametrize("G,R,mod,vmod", [(1, 1, None, None), (1, 2, 3, 2), (1, 100, 10, 3),
                                          (1, 5000, 50, 4), (1, 100000, None, None),
                                          (4, 3000, 7, 2), (257, 17, 5, 2), (3, 2049, 2, 2)])
def test_lww_lub_many(gpu_ctx, G, R, mod, vmod):
    m, v = _inputs(0x5EED0004 + R, G, R, mod, vmod)
    res = cg.lwwreg.lub_many(to_dev(m), to_dev(v), ctx=gpu_ctx)
    gm, gv, gf = (to_host(t) for t in res)
    for g in range(G):
        om, ov, of, _ = O.lwwreg_fold(m[g], v[g])
        assert (int(gm[g]), int(gv[g]), int(gf[g])) == (om, ov, of), g


def test_lww_no_conflicts_when_markers_unique(gpu_ctx):
    R = 10000
    m = np.random.default_rng(1).permutation(R).astype(np.uint64)
    v = O.synth_matrix(2, 1, R, 3)[0]
    res = cg.lwwreg.lub_many(to_dev(m), to_dev(v), ctx=gpu_ctx)
    assert int(to_host(res.marker)) == R - 1
    assert int(to_host(res.val)) == int(v[np.argmax(m)])
    assert to_host(res.first_conflict) == NONE


@pytest.mark.parametrize("N", [1, 77, 4096])
def test_lww_merge_batch(gpu_ctx, N):
    sm, sv = _inputs(21, 1, N, 4, 2)
    om, ov = _inputs(22, 1, N, 4, 2)
    sm, sv, om, ov = sm[0], sv[0], om[0], ov[0]
    dsm, dsv = to_dev(sm), to_dev(sv)
    conflict = cg.lwwreg.merge_batch(dsm, dsv, to_dev(om), to_dev(ov), ctx=gpu_ctx)
    gm, gv = to_host(dsm), to_host(dsv)
    gc = conflict.cpu().numpy()
    for i in range(N):
        reg = O.LWWReg(int(sv[i]), int(sm[i]))
        try:
            reg.merge(O.LWWReg(int(ov[i]), int(om[i])))
            err = 0
        except O.ConflictingMarker:
            err = 1
        assert (int(gm[i]), int(gv[i]), int(gc[i])) == (reg.marker, reg.val, err)


@pytest.mark.parametrize("G,R,split", [(1, 5000, 1234), (3, 700, 350), (2, 9000, 8999), (1, 10, 0)])
def test_lww_accumulate_continues_the_fold(gpu_ctx, G, R, split):
    """lub of the tail continued from the lub of the head == lub of everything, and the tail's
    conflict index + split == the global first conflict when the head has none."""
    m, v = _inputs(0x77 + R, G, R, 9, 2)
    dm, dv = to_dev(m), to_dev(v)
    full = cg.lwwreg.lub_many(dm, dv, ctx=gpu_ctx)
    if split == 0:
        init = (dm[:, 0].contiguous(), dv[:, 0].contiguous())
        tail = cg.lwwreg.lub_many(dm[:, 1:].contiguous(), dv[:, 1:].contiguous(), ctx=gpu_ctx, init=init)
        off = 1
        head_fc = np.full(G, NONE)
    else:
        head = cg.lwwreg.lub_many(dm[:, :split].contiguous(), dv[:, :split].contiguous(), ctx=gpu_ctx)
        tail = cg.lwwreg.lub_many(dm[:, split:].contiguous(), dv[:, split:].contiguous(), ctx=gpu_ctx,
                                  init=(head.marker, head.val))
        off = split
        head_fc = to_host(head.first_conflict)
    np.testing.assert_array_equal(to_host(tail.marker), to_host(full.marker))
    np.testing.assert_array_equal(to_host(tail.val), to_host(full.val))
    tfc = to_host(tail.first_conflict)
    ffc = to_host(full.first_conflict)
    for g in range(G):
        exp = head_fc[g] if head_fc[g] != NONE else (NONE if tfc[g] == NONE else tfc[g] + np.uint64(off))
        assert ffc[g] == exp
