"""Replay the reference's known-answer tests with every merge executed by libcrdt_gpu:
reference-shaped states are interned to the dense layout, merged on the GPU and egressed.  Two
routes per merge: a 2-replica lub_many (acc = new(); acc.merge(self); acc.merge(other)) and the
in-place pairwise merge_batch (self.merge(other) itself, N = 1)."""
import numpy as np
import pytest
import torch

import kat_runner as K
import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import intern  # noqa: E402


def _vc_pair(a: O.VClock, b: O.VClock, idx):
    rows = intern.clocks_to_dense([a.dots, b.dots], idx)
    return rows


def _pair_merge(mod, rows, mode):
    """rows (2, W) -> merged row: lub_many of the 2 replicas, or merge_batch of self=row 0."""
    d = to_dev(rows)
    if mode == "lub2":
        return to_host(mod.lub_many(d))
    me = d[:1].clone()
    mod.merge_batch(me, d[1:])
    return to_host(me)[0]


def gpu_merge(dst, src, kind, mode="lub2"):
    if kind in ("vclock", "gcounter"):
        da = dst if kind == "vclock" else dst.inner
        sa = src if kind == "vclock" else src.inner
        idx = intern.Index()
        rows = _vc_pair(da, sa, idx)
        out = _pair_merge(cg.vclock if kind == "vclock" else cg.gcounter, rows, mode)
        da.dots = intern.dense_to_clocks(out[None, :], idx)[0]
        return dst
    if kind == "pncounter":
        idx = intern.Index()
        p = intern.clocks_to_dense([dst.p.inner.dots, src.p.inner.dots], idx)
        n = intern.clocks_to_dense([dst.n.inner.dots, src.n.inner.dots], idx, width=p.shape[1])
        p = np.pad(p, ((0, 0), (0, n.shape[1] - p.shape[1])))
        out = _pair_merge(cg.pncounter, np.concatenate([p, n], axis=1), mode)
        A = p.shape[1]
        dst.p.inner.dots = intern.dense_to_clocks(out[None, :A], idx)[0]
        dst.n.inner.dots = intern.dense_to_clocks(out[None, A:], idx)[0]
        return dst
    if kind == "gset":
        idx = intern.Index()
        bm = intern.sets_to_bitmap([dst.value, src.value], idx)
        out = _pair_merge(cg.gset, bm, mode)
        dst.value = intern.bitmap_to_sets(out[None, :], idx)[0]
        return dst
    if kind == "lwwreg":
        vals = intern.Index([dst.val, src.val])
        m = to_dev(np.array([dst.marker, src.marker], dtype=np.uint64))
        v = to_dev(np.array([vals.pos[dst.val], vals.pos[src.val]], dtype=np.uint64))
        conflict = cg.lwwreg.merge_batch(m[:1].clone(), v[:1].clone(), m[1:], v[1:])
        if int(conflict.cpu()[0]):
            raise O.ConflictingMarker()
        res = cg.lwwreg.lub_many(m, v)
        dst.marker, dst.val = int(to_host(res.marker)), vals.ids[int(to_host(res.val))]
        return dst
    if kind == "orswot":
        return gpu_orswot_merge(dst, src) if mode == "lub2" else gpu_orswot_merge_batch(dst, src)
    raise TypeError(kind)


def gpu_orswot_merge_batch(dst: O.Orswot, src: O.Orswot) -> O.Orswot:
    """dst.merge(src) as crdt_orswot_merge_batch with N = 1 (in place on dst's dense state)."""
    from orswot_apply_util import dense_states, to_object
    actors, members = intern.Index(), intern.Index()
    for s in (dst, src):
        for a in s.clock.dots:
            actors.intern(a)
        for m, c in s.entries.items():
            members.intern(m)
            for a in c.dots:
                actors.intern(a)
        for k, ms in s.deferred.items():
            for a in k.dots:
                actors.intern(a)
            for m in ms:
                members.intern(m)
    A, M = max(1, len(actors)), max(1, len(members))
    fa, fm = (lambda a: actors.pos[a]), (lambda m: members.pos[m])
    from orswot_apply_util import map_orswot
    Dcap = max(1, len(dst.deferred) + len(src.deferred))
    sides = []
    for s in (dst, src):
        c, e, dc, dm, n = dense_states([map_orswot(s, fa, fm)], M, A, Dcap)
        sides.append(cg.orswot.OrswotStates(to_dev(c), to_dev(e), to_dev(dc), to_dev(dm),
                                            torch.from_numpy(n.astype(np.int32)).cuda()))
    status = cg.orswot.merge_batch(sides[0], sides[1]).cpu().numpy()
    assert status[0] == 0, status
    me = sides[0]
    dense = to_object(to_host(me.clock), to_host(me.entries), to_host(me.def_clock), to_host(me.def_members),
                      me.def_count.cpu().numpy(), 0)
    return map_orswot(dense, lambda a: actors.ids[a], lambda m: members.ids[m])


def gpu_orswot_merge(dst: O.Orswot, src: O.Orswot) -> O.Orswot:
    actors, members = intern.Index(), intern.Index()
    states = [dst, src]
    for s in states:
        for a in s.clock.dots:
            actors.intern(a)
        for m, c in s.entries.items():
            members.intern(m)
            for a in c.dots:
                actors.intern(a)
        for k, ms in s.deferred.items():
            for a in k.dots:
                actors.intern(a)
            for m in ms:
                members.intern(m)
    A, M = max(1, len(actors)), max(1, len(members))
    Mw = (M + 63) // 64
    clock = np.zeros((2, A), dtype=np.uint64)
    entries = np.zeros((2, M, A), dtype=np.uint64)
    dcl, dmem = [], []
    for r, s in enumerate(states):
        for a, v in s.clock.dots.items():
            clock[r, actors.pos[a]] = v
        for m, c in s.entries.items():
            for a, v in c.dots.items():
                entries[r, members.pos[m], actors.pos[a]] = v
        for k, ms in s.deferred.items():
            row = np.zeros(A, dtype=np.uint64)
            for a, v in k.dots.items():
                row[actors.pos[a]] = v
            bits = np.zeros(Mw, dtype=np.uint64)
            for m in ms:
                p = members.pos[m]
                bits[p // 64] |= np.uint64(1) << np.uint64(p % 64)
            dcl.append(row)
            dmem.append(bits)
    D = len(dcl)
    kw = {}
    if D:
        kw = dict(def_off=[0, D], def_clock=to_dev(np.stack(dcl)), def_members=to_dev(np.stack(dmem)))
    res = cg.orswot.lub_many(to_dev(clock), to_dev(entries), **kw)
    c, e = to_host(res.clock), to_host(res.entries)
    out = O.Orswot()
    out.clock = O.VClock({actors.ids[a]: int(v) for a, v in enumerate(c) if v and a < len(actors)})
    for m in range(len(members)):
        row = e[m]
        if row.any():
            out.entries[members.ids[m]] = O.VClock({actors.ids[a]: int(v) for a, v in enumerate(row) if v})
    if D:
        for rm, ms in cg.orswot.deferred_set(kw["def_clock"], res.def_keep, res.def_members):
            k = O.VClock({actors.ids[a]: v for a, v in enumerate(rm) if v})
            out.deferred[k] = {members.ids[m] for m in ms}
    return out


CASES = [c for f in ("kat_vclock.json", "kat_counters.json", "kat_orswot.json")
         for c in K.load_cases(f) if any(s[0] in ("merge", "merge_err") for s in c["steps"])]


@pytest.mark.parametrize("mode", ["lub2", "merge_batch"])
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_kat_gpu(gpu_ctx, case, mode):
    K.run_case(case, merge_hook=lambda d, s, k: gpu_merge(d, s, k, mode))


class GpuCausal:
    """Routes the KATs' VClock forget / glb / partial_cmp and counter read() through
    libcrdt_gpu (crdt_vclock_pair_op, crdt_vclock_partial_cmp, crdt_*counter_read)."""

    CODES = {0: O.EQUAL, 1: O.GREATER, -1: O.LESS, 2: O.NONE}

    def _pair(self, x, y):
        idx = intern.Index()
        rows = intern.clocks_to_dense([x.dots, y.dots], idx)
        return idx, to_dev(rows)

    def forget(self, x, y):
        idx, d = self._pair(x, y)
        out = to_host(cg.causal.forget(d[0], d[1]))
        x.dots = intern.dense_to_clocks(out[None, :], idx)[0]

    def glb(self, x, y):
        idx, d = self._pair(x, y)
        out = to_host(cg.causal.glb(d[0], d[1]))
        x.dots = intern.dense_to_clocks(out[None, :], idx)[0]

    def cmp(self, x, y):
        _, d = self._pair(x, y)
        return self.CODES[int(cg.causal.partial_cmp(d[0], d[1]).cpu())]

    def read(self, v):
        idx = intern.Index()
        if isinstance(v, O.GCounter):
            rows = intern.clocks_to_dense([v.inner.dots], idx)
            return cg.gcounter.read(to_dev(rows[0]))
        p = intern.clocks_to_dense([v.p.inner.dots], idx)
        n = intern.clocks_to_dense([v.n.inner.dots], idx, width=p.shape[1])
        p = np.pad(p, ((0, 0), (0, n.shape[1] - p.shape[1])))
        return cg.pncounter.read(to_dev(np.concatenate([p, n], axis=1)[0]))


CAUSAL_CASES = [c for f in ("kat_vclock.json", "kat_counters.json") for c in K.load_cases(f)
                if any(s[0] in ("forget", "glb", "assert_cmp", "assert_read") for s in c["steps"])]


@pytest.mark.parametrize("case", CAUSAL_CASES, ids=[c["name"] for c in CAUSAL_CASES])
def test_kat_gpu_causal(gpu_ctx, case):
    """The reference's KATs with merges AND forget / glb / partial_cmp / read on the GPU."""
    K.run_case(case, merge_hook=gpu_merge, causal_hook=GpuCausal())
