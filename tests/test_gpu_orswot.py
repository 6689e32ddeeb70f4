"""GPU parity: Orswot lub_many vs the oracle fold (reference semantics incl. deferred removes)."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _run(gpu_ctx, clock, entries, off, dcl, dmem):
    R, M, A = entries.shape
    D = dcl.shape[0]
    kw = {}
    if D:
        kw = dict(def_off=[0, D], def_clock=to_dev(dcl), def_members=to_dev(dmem))
    res = cg.orswot.lub_many(to_dev(clock), to_dev(entries), ctx=gpu_ctx, **kw)
    c, e = to_host(res.clock), to_host(res.entries)
    d = cg.orswot.deferred_set(kw["def_clock"], res.def_keep, res.def_members) if D else set()
    return c, e, d


@pytest.mark.parametrize("seed,R,M,A", [(1, 1, 1, 1), (2, 2, 5, 3), (3, 9, 40, 6), (4, 33, 64, 8),
                                        (5, 64, 200, 16), (6, 300, 128, 64), (7, 20, 70, 33),
                                        (8, 1000, 16, 4)])
def test_orswot_lub_many(gpu_ctx, seed, R, M, A):
    clock, entries, off, dcl, dmem = O.gen_orswot(seed, R, M, A, kmax=16)
    oc, oe, odef, _ = O.orswot_fold(clock, entries, off, dcl, dmem)
    c, e, d = _run(gpu_ctx, clock, entries, off, dcl, dmem)
    np.testing.assert_array_equal(c, oc)
    np.testing.assert_array_equal(e, oe)
    assert d == odef


def test_orswot_groups(gpu_ctx):
    G, R, M, A = 3, 12, 50, 8
    parts = [O.gen_orswot(40 + g, R, M, A, kmax=10) for g in range(G)]
    clock = np.stack([p[0] for p in parts])
    entries = np.stack([p[1] for p in parts])
    dcl = np.concatenate([p[3] for p in parts])
    dmem = np.concatenate([p[4] for p in parts])
    off = np.cumsum([0] + [p[3].shape[0] for p in parts])
    res = cg.orswot.lub_many(to_dev(clock), to_dev(entries), def_off=off, def_clock=to_dev(dcl),
                             def_members=to_dev(dmem), ctx=gpu_ctx)
    gc, ge = to_host(res.clock), to_host(res.entries)
    for g, p in enumerate(parts):
        oc, oe, odef, _ = O.orswot_fold(*p)
        np.testing.assert_array_equal(gc[g], oc)
        np.testing.assert_array_equal(ge[g], oe)
        got = cg.orswot.deferred_set(to_dev(dcl), res.def_keep, res.def_members, int(off[g]), int(off[g + 1]))
        assert got == odef


def test_orswot_duplicate_deferred_union(gpu_ctx):
    """Two replicas holding the same future rm clock over different members: one survivor with
    the union of the member sets (orswot.rs:242-246)."""
    A, M = 4, 8
    clock = np.array([[1, 0, 0, 0], [0, 2, 0, 0]], dtype=np.uint64)
    entries = np.zeros((2, M, A), dtype=np.uint64)
    entries[0, 1, 0] = 1
    entries[1, 2, 1] = 2
    rm = np.array([0, 0, 5, 0], dtype=np.uint64)
    dcl = np.stack([rm, rm, np.array([1, 1, 0, 0], dtype=np.uint64)])
    dmem = np.array([[1 << 3], [1 << 4], [1 << 1]], dtype=np.uint64)
    off = np.array([0, 1, 3], dtype=np.uint64)
    oc, oe, odef, _ = O.orswot_fold(clock, entries, off, dcl, dmem)
    c, e, d = _run(gpu_ctx, clock, entries, off, dcl, dmem)
    assert d == odef == {((0, 0, 5, 0), frozenset({3, 4}))}
    np.testing.assert_array_equal(e, oe)


def test_orswot_empty_and_idempotent(gpu_ctx):
    clock, entries, off, dcl, dmem = O.gen_orswot(9, 10, 30, 6, kmax=8, p_def=0.0)
    res = cg.orswot.lub_many(to_dev(clock), to_dev(entries), ctx=gpu_ctx)
    # lub of the lub with itself (and with the inputs again) changes nothing
    twice = cg.orswot.lub_many(torch.stack([res.clock, res.clock]), torch.stack([res.entries, res.entries]), ctx=gpu_ctx)
    assert torch.equal(twice.clock, res.clock) and torch.equal(twice.entries, res.entries)
    none = cg.orswot.lub_many(torch.empty((0, 6), dtype=torch.int64, device="cuda:0"),
                              torch.empty((0, 30, 6), dtype=torch.int64, device="cuda:0"), ctx=gpu_ctx)
    assert int(none.clock.abs().sum()) == 0 and int(none.entries.abs().sum()) == 0


def test_synth_orswot_matches_cpu(gpu_ctx):
    from crdts_gpu import synth
    R, M, A, kmax = 37, 130, 12, 40
    inp = synth.orswot_replicas(gpu_ctx, R, M, A, seed=77, kmax=kmax, first_row=5, p_def=0.3)
    c, e = O.synth_orswot(77, R, M, A, kmax, row0=5)
    rows = np.repeat(np.arange(R), np.diff(inp.def_off.astype(np.int64)))
    e = O.apply_rm_rows(e, rows, to_host(inp.def_clock), to_host(inp.def_members))
    np.testing.assert_array_equal(to_host(inp.clock), c)
    np.testing.assert_array_equal(to_host(inp.entries), e)


@pytest.mark.parametrize("R,M,A", [(512, 300, 64), (2000, 64, 16), (129, 1000, 8)])
def test_orswot_lub_many_synth(gpu_ctx, R, M, A):
    from crdts_gpu import synth
    inp = synth.orswot_replicas(gpu_ctx, R, M, A, seed=R + M, kmax=min(M - 1, 30), p_def=0.1)
    D = inp.def_clock.shape[0]
    res = cg.orswot.lub_many(inp.clock, inp.entries, def_off=[0, D], def_clock=inp.def_clock,
                             def_members=inp.def_members, ctx=gpu_ctx)
    oc, oe, odef, _ = O.orswot_fold(to_host(inp.clock), to_host(inp.entries), inp.def_off,
                                    to_host(inp.def_clock), to_host(inp.def_members))
    np.testing.assert_array_equal(to_host(res.clock), oc)
    np.testing.assert_array_equal(to_host(res.entries), oe)
    assert cg.orswot.deferred_set(inp.def_clock, res.def_keep, res.def_members) == odef


def _witness_states(seed, i, n_ops=40):
    """test/orswot.rs:33-68: random Add/Rm ops routed by actor % i to i witnesses."""
    rng = np.random.default_rng(seed)
    ops = []
    for _ in range(n_ops):
        actor = int(rng.integers(0, 11))
        members = set(int(x) for x in rng.integers(0, 8, size=int(rng.integers(1, 4))))
        counter = int(rng.integers(1, 9))
        if rng.integers(0, 2) == 0:
            ops.append((actor, O.OrswotAdd(O.Dot(actor, counter), members)))
        else:
            ops.append((actor, O.OrswotRm(O.VClock({actor: counter}), members)))
    w = [O.Orswot() for _ in range(i)]
    for a, op in ops:
        w[a % i].apply(op)
    return w


def _dense(ws, A=11, M=8):
    R = len(ws)
    clock = np.zeros((R, A), np.uint64)
    ent = np.zeros((R, M, A), np.uint64)
    dcl, dm, off = [], [], [0]
    for r, w in enumerate(ws):
        for a, v in w.clock.dots.items():
            clock[r, a] = v
        for m, c in w.entries.items():
            for a, v in c.dots.items():
                ent[r, m, a] = v
        for k, ms in w.deferred.items():
            row = np.zeros(A, np.uint64)
            for a, v in k.dots.items():
                row[a] = v
            bits = np.zeros(1, np.uint64)
            for m in ms:
                bits[0] |= np.uint64(1) << np.uint64(m)
            dcl.append(row)
            dm.append(bits)
        off.append(len(dcl))
    return clock, ent, np.array(off, np.uint64), np.array(dcl, np.uint64).reshape(-1, A), np.array(dm, np.uint64).reshape(-1, 1)


@pytest.mark.parametrize("seed", range(12))
def test_orswot_witness_convergence_gpu(gpu_ctx, seed):
    """prop_merge_converges on the GPU: for i in 2..11 witnesses the GPU lub equals the
    reference fold (oracle) — and is identical when run twice (determinism)."""
    for i in range(2, 11):
        ws = _witness_states(seed, i)
        clock, ent, off, dcl, dm = _dense(ws)
        oc, oe, odef, _ = O.orswot_fold(clock, ent, off, dcl, dm)
        for _rep in range(2):
            c, e, d = _run(gpu_ctx, clock, ent, off, dcl, dm)
            assert np.array_equal(c, oc), (seed, i, "clock")
            assert np.array_equal(e, oe), (seed, i, "entries", np.argwhere(e != oe)[:4])
            assert d == odef, (seed, i, d, odef)


def _many_groups(G, seed, R=4, M=64, A=8, per_group=16):
    """G groups of well-formed replicas, each group with `per_group` future removes drawn from 4
    distinct rm clocks (so many survivors share a clock and their member sets must merge), held
    by replicas in order and pre-applied (apply_rm, orswot.rs:230-238)."""
    rng = np.random.default_rng(seed)
    parts = []
    for g in range(G):
        clock, entries, _, _, _ = O.gen_orswot(seed * 100003 + g, R, M, A, kmax=10, p_def=0.0)
        top = clock.max(axis=0)
        pats = []
        for _ in range(4):
            rm = top // np.uint64(2)
            rm[int(rng.integers(0, A))] = top.max() + np.uint64(1 + int(rng.integers(0, 2)))
            pats.append(rm)
        rows = np.sort(rng.integers(0, R, size=per_group))
        dcl = np.stack([pats[int(rng.integers(0, 4))] for _ in rows])
        dmem = np.zeros((per_group, 1), np.uint64)
        for d, r in enumerate(rows):
            for m in rng.choice(M, size=2, replace=False):
                dmem[d, 0] |= np.uint64(1) << np.uint64(m)
                row = entries[r, m]
                row[row <= dcl[d]] = 0
        off = np.searchsorted(rows, np.arange(R + 1)).astype(np.uint64)
        parts.append((clock, entries, off, dcl, dmem))
    return parts


def _run_groups(ctx, parts):
    clock = np.stack([p[0] for p in parts])
    entries = np.stack([p[1] for p in parts])
    dcl = np.concatenate([p[3] for p in parts])
    dmem = np.concatenate([p[4] for p in parts])
    off = np.cumsum([0] + [p[3].shape[0] for p in parts])
    args = (to_dev(clock), to_dev(entries))
    kw = dict(def_off=off, def_clock=to_dev(dcl), def_members=to_dev(dmem), ctx=ctx)
    cg.orswot.lub_many(*args, **kw)  # warm
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    res = cg.orswot.lub_many(*args, **kw)
    torch.cuda.synchronize()
    return res, off, dcl, time.perf_counter() - t0


def test_orswot_many_groups_deferred_dedup(gpu_ctx):
    """>= 1,000 groups x 16 deferred removes each: every group's survivors (identical clocks merged)
    equal the oracle fold's, and the dedup is linear in the survivors: 4x the groups costs far
    less than the 16x a whole-list scan per survivor would."""
    parts = _many_groups(1000, 7)
    res, off, dcl, t1 = _run_groups(gpu_ctx, parts)
    gc, ge = to_host(res.clock), to_host(res.entries)
    merged = 0
    for g, p in enumerate(parts):
        oc, oe, odef, _ = O.orswot_fold(*p)
        np.testing.assert_array_equal(gc[g], oc)
        np.testing.assert_array_equal(ge[g], oe)
        got = cg.orswot.deferred_set(to_dev(dcl), res.def_keep, res.def_members, int(off[g]), int(off[g + 1]))
        assert got == odef, g
        merged += 16 - len(odef)
    assert merged > 1000  # identical clocks really merged
    _, _, _, t4 = _run_groups(gpu_ctx, _many_groups(4000, 8))
    assert t4 < 8 * t1 + 0.002, (t1, t4)
