"""MVReg<u64, A> on its own through libcrdt_gpu (crdt_mvreg_lub_many / _merge_batch / _apply_batch,
csrc/mvreg.hip) against the reference's semantics:

  * the reference's own MVReg tests (test/mvreg.rs:11-105, the doctest at src/mvreg.rs:13-31),
    transcribed as step scripts (tests/golden/kat_mvreg.json), replayed with EVERY merge and EVERY
    apply executed on the GPU (merge both as a 2-replica lub_many and as merge_batch);
  * random registers against the oracle's restated MVReg::merge / apply (oracle/oracle.py,
    mvreg.rs:112-166): left folds, pairwise merges, op streams incl. empty-clock Puts, dominated
    and concurrent writes, and the capacity status bits; A up to 200 (1, 2 and 4 clock words per
    lane)."""
import numpy as np
import pytest
import torch

import kat_runner as K
import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import intern  # noqa: E402


def dense_regs(regs, actors, V, vals):
    """MVReg objects -> (vclk (N, V, A), vval (N, V)) with values interned into `vals`."""
    A = max(1, len(actors.ids))
    vc = np.zeros((len(regs), V, A), np.uint64)
    vv = np.zeros((len(regs), V), np.uint64)
    for i, r in enumerate(regs):
        assert len(r.vals) <= V
        for s, (c, v) in enumerate(r.vals):
            for a, k in c.dots.items():
                vc[i, s, actors.intern(a)] = k
            vv[i, s] = vals.intern(v)
    return vc, vv


def obj_regs(vc, vv, actors, vals, n=None):
    out = []
    for i in range(vc.shape[0]):
        r = O.MVReg()
        for s in range(vc.shape[1] if n is None else int(n[i])):
            row = vc[i, s]
            if not row.any():
                continue
            r.vals.append((O.VClock({actors.ids[a]: int(row[a]) for a in np.flatnonzero(row)}), vals.ids[int(vv[i, s])]))
        out.append(r)
    return out


def _index_of(*regs_or_ops):
    actors = intern.Index()
    for x in regs_or_ops:
        clocks = [c for c, _ in x.vals] if isinstance(x, O.MVReg) else [x.clock]
        for c in clocks:
            for a in sorted(c.dots, key=str):
                actors.intern(a)
    return actors


def gpu_merge(dst, src, mode):
    actors, vals = _index_of(dst, src), intern.Index()
    if mode == "lub2":
        V = max(1, len(dst.vals), len(src.vals))
        vc, vv = dense_regs([dst, src], actors, V, vals)
        res = cg.mvreg.lub_many(to_dev(vc), to_dev(vv), vout=max(4, len(dst.vals) + len(src.vals)))
        got = obj_regs(to_host(res.vclk)[None], to_host(res.vval)[None], actors, vals, res.nval.cpu().numpy())[0]
    else:
        V = len(dst.vals) + len(src.vals) + 1
        svc, svv = dense_regs([dst], actors, V, vals)
        ovc, ovv = dense_regs([src], actors, max(1, len(src.vals)), vals)
        s_c, s_v = to_dev(svc), to_dev(svv)
        st = cg.mvreg.merge_batch(s_c, s_v, to_dev(ovc), to_dev(ovv))
        assert int(st.cpu()[0]) == 0
        got = obj_regs(to_host(s_c), to_host(s_v), actors, vals)[0]
    dst.vals = got.vals
    return dst


def gpu_apply(reg, op):
    if not isinstance(reg, O.MVReg):
        return reg.apply(op)
    actors, vals = _index_of(reg, op), intern.Index()
    V = len(reg.vals) + 1
    vc, vv = dense_regs([reg], actors, V, vals)
    A = vc.shape[2]
    row = np.zeros(A, np.uint64)
    for a, k in op.clock.dots.items():
        row[actors.intern(a)] = k
    ops = cg.mvreg.encode_ops([[(row, vals.intern(op.val))]], A, "cuda")
    d_c, d_v = to_dev(vc), to_dev(vv)
    st = cg.mvreg.apply_batch(d_c, d_v, ops)
    assert int(st.cpu()[0]) == 0
    reg.vals = obj_regs(to_host(d_c), to_host(d_v), actors, vals)[0].vals


@pytest.mark.parametrize("mode", ["lub2", "merge_batch"])
@pytest.mark.parametrize("case", K.load_cases("kat_mvreg.json"), ids=lambda c: c["name"])
def test_kat_mvreg_on_gpu(gpu_ctx, case, mode):
    hook = lambda d, s, kind: gpu_merge(d, s, mode) if kind == "mvreg" else K.default_merge(d, s, kind)  # noqa: E731
    K.run_case(case, merge_hook=hook, apply_hook=gpu_apply)


# ---- random registers vs the oracle ---------------------------------------------------------------
def rand_regs(rng, n, A, nact, vmax, steps=6, group=None):
    """Registers built by random Puts whose clocks advance random actors (so values are concurrent,
    dominated or equal as the history goes). With `group`, every run of `group` registers shares one
    advancing causal history, so a group's fold keeps a bounded number of concurrent values."""
    regs = []
    for i in range(n):
        r = O.MVReg()
        if group is None or i % group == 0:
            base = O.VClock()
        for _ in range(rng.integers(0, steps + 1)):
            c = base.copy()
            for a in rng.choice(nact, size=rng.integers(1, 3), replace=False):
                c.apply(O.Dot(int(a), int(rng.integers(1, 6))))
            if rng.random() < 0.5:
                base = c.copy()
            r.apply(O.MVRegPut(c, int(rng.integers(0, 2**63))))
            if len(r.vals) > vmax:
                r.vals = r.vals[:vmax]
        regs.append(r)
    return regs


@pytest.mark.parametrize("A", [5, 64, 100, 200])
def test_mvreg_lub_many_vs_oracle(gpu_ctx, A):
    rng = np.random.default_rng(A)
    G, R, V = 7, 40, 4
    regs = rand_regs(rng, G * R, A, min(A, 8), V, group=13)
    actors = intern.Index(list(range(A)))
    vals = intern.Index()
    vc, vv = dense_regs(regs, actors, V, vals)
    folds = []
    for g in range(G):
        acc = O.MVReg()
        for r in regs[g * R:(g + 1) * R]:
            acc.merge(r)
        folds.append(acc)
    assert max(len(f.vals) for f in folds) <= 16  # the generator keeps every fold within vout
    res = cg.mvreg.lub_many(to_dev(vc.reshape(G, R, V, A)), to_dev(vv.reshape(G, R, V)), vout=16)
    got = obj_regs(to_host(res.vclk), to_host(res.vval), actors, vals, res.nval.cpu().numpy())
    for g in range(G):
        assert got[g].vals == folds[g].vals  # same values in the same Vec order


def test_mvreg_lub_many_capacity_and_empty(gpu_ctx):
    """Twelve concurrent writers: vout=8 raises, vout=16 holds all twelve in the reference's order;
    R = 0 folds to the empty register."""
    A = 12
    regs = []
    for a in range(A):
        regs.append(O.MVReg([(O.VClock({a: 1}), 100 + a)]))
    actors, vals = intern.Index(list(range(A))), intern.Index()
    vc, vv = dense_regs(regs, actors, 1, vals)
    with pytest.raises(cg.mvreg.MVRegCapacityError):
        cg.mvreg.lub_many(to_dev(vc), to_dev(vv), vout=8)
    res = cg.mvreg.lub_many(to_dev(vc), to_dev(vv), vout=16)
    acc = O.MVReg()
    for r in regs:
        acc.merge(r)
    got = obj_regs(to_host(res.vclk)[None], to_host(res.vval)[None], actors, vals, res.nval.cpu().numpy())[0]
    assert got.vals == acc.vals and len(got.vals) == 12
    empty = cg.mvreg.lub_many(to_dev(vc[:0]), to_dev(vv[:0]), vout=2)
    assert int(empty.nval.cpu()[0]) == 0 and not to_host(empty.vclk).any()


@pytest.mark.parametrize("A", [7, 130])
def test_mvreg_merge_batch_vs_oracle(gpu_ctx, A):
    rng = np.random.default_rng(100 + A)
    N, V = 300, 3
    a_regs = rand_regs(rng, N, A, min(A, 6), V)
    b_regs = rand_regs(rng, N, A, min(A, 6), V)
    actors, vals = intern.Index(list(range(A))), intern.Index()
    svc, svv = dense_regs(a_regs, actors, 2 * V, vals)
    ovc, ovv = dense_regs(b_regs, actors, V, vals)
    s_c, s_v = to_dev(svc), to_dev(svv)
    st = cg.mvreg.merge_batch(s_c, s_v, to_dev(ovc), to_dev(ovv))
    assert (st.cpu().numpy() == 0).all()
    got = obj_regs(to_host(s_c), to_host(s_v), actors, vals)
    for i in range(N):
        exp = a_regs[i].copy()
        exp.merge(b_regs[i])
        assert got[i].vals == exp.vals, i
    # self's slots too small for the merged register: status bit 4
    s2c, s2v = to_dev(svc[:, :1].copy()), to_dev(svv[:, :1].copy())
    st = cg.mvreg.merge_batch(s2c, s2v, to_dev(ovc), to_dev(ovv)).cpu().numpy()
    need = np.array([len(O.MVReg(a.vals[:1]).vals) for a in a_regs])
    for i in range(N):
        exp = O.MVReg(a_regs[i].vals[:1])
        exp.merge(b_regs[i])
        assert bool(st[i] & 16) == (len(exp.vals) > 1), (i, need[i])


@pytest.mark.parametrize("A", [6, 90, 256])
def test_mvreg_apply_batch_vs_oracle(gpu_ctx, A):
    rng = np.random.default_rng(200 + A)
    N, V = 200, 6
    regs = rand_regs(rng, N, A, min(A, 5), 2)
    streams, exp = [], []
    for r in regs:
        e = r.copy()
        ops = []
        for _ in range(rng.integers(0, 9)):
            c = e.clock() if rng.random() < 0.6 else O.VClock()
            c = c.copy()
            if rng.random() < 0.85:  # an empty clock (no-op) otherwise
                for a in rng.choice(min(A, 5), size=rng.integers(1, 3), replace=False):
                    c.apply(O.Dot(int(a), c.get(int(a)) + int(rng.integers(0, 3))))
            v = int(rng.integers(0, 1000))
            ops.append((c, v))
            e.apply(O.MVRegPut(c, v))
        streams.append(ops)
        exp.append(e)
    actors, vals = intern.Index(list(range(A))), intern.Index()
    vc, vv = dense_regs(regs, actors, V, vals)
    enc = [[({a: k for a, k in c.dots.items()}, vals.intern(v)) for c, v in ops] for ops in streams]
    d_c, d_v = to_dev(vc), to_dev(vv)
    st = cg.mvreg.apply_batch(d_c, d_v, cg.mvreg.encode_ops(enc, A, "cuda")).cpu().numpy()
    got = obj_regs(to_host(d_c), to_host(d_v), actors, vals)
    for i in range(N):
        if len(exp[i].vals) <= V:
            assert st[i] == 0 and got[i].vals == exp[i].vals, i
        else:
            assert st[i] & 16, i
