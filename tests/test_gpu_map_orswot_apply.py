"""GPU: CmRDT::apply of Map<K, Orswot<M>> (round 5; crdt_map_orswot_apply_batch) against the oracle's
Map.apply (map.rs:119-137) with Orswot::apply (orswot.rs:55-79, apply_rm :230-250, apply_deferred
:281-286) inside and the Map's apply_keyset_rm / apply_deferred (:311-348, Orswot::forget :150-183):
op-replay states folded alone, then streams of Orswot Adds (fresh / seen dots), Orswot Rms (clocks
from the future: nested deferred removes, re-applied by later Adds), Map Rms (deferred at the Map
level, re-applied by later Ups), at A within and past one lane word and M past 64."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _states(ctx, maps, K, M, A):
    N = len(maps)
    d = O.map_orswot_to_dense(maps, K, M, A)
    D = d["def_row"].shape[0]
    off = [0]
    for m in maps:
        off.append(off[-1] + len(m.deferred))
    kw = dict(def_off=off, def_row=torch.zeros(D, dtype=torch.int32, device="cuda:0"),
              def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"])) if D else {}
    Dv = int(d["vd_off"][-1])
    vkw = dict(vd_clock=to_dev(d["vd_clock"]), vd_mem=to_dev(d["vd_members"])) if Dv else {}
    shp = lambda x: to_dev(x.reshape((N, 1) + x.shape[1:]))  # noqa: E731
    res = cg.map.orswot_lub_many(shp(d["clock"]), shp(d["ec"]), shp(d["oc"]), shp(d["ent"]), to_dev(d["vd_off"]),
                                 ctx=ctx, **vkw, **kw)
    return res, kw, off


def _streams(rng, exps, K, M, A, T):
    streams, oops = [], []
    for m in exps:
        clk = {a: m.clock.get(a) for a in range(A)}
        occ = {}  # the Orswot clocks the stream has seen (per key), for fresh / seen nested dots
        for k, e in m.entries.items():
            occ[k] = {a: e.val.clock.get(a) for a in range(A)}
        ops, oo = [], []
        for _ in range(T):
            x = rng.random()
            if x < 0.8:
                a = int(rng.integers(A))
                c = clk[a] + int(rng.integers(1, 3)) if rng.random() < 0.85 else max(clk[a] - int(rng.integers(0, 2)), 1)
                clk[a] = max(clk[a], c)
                k = int(rng.integers(K))
                oc = occ.setdefault(k, {a2: 0 for a2 in range(A)})
                ms = sorted(set(int(z) for z in rng.choice(M, size=int(rng.integers(1, 3)), replace=False)))
                if rng.random() < 0.65:  # Orswot Add
                    va = int(rng.integers(A))
                    vc = oc[va] + int(rng.integers(1, 3)) if rng.random() < 0.85 else max(oc[va], 1)
                    oc[va] = max(oc[va], vc)
                    ops.append(("add", a, c, k, va, vc, ms))
                    oo.append(O.MapUp(O.Dot(a, c), k, O.OrswotAdd(O.Dot(va, vc), ms)))
                else:  # Orswot Rm, its clock up to 2 ahead of the seen Orswot clock on some actors
                    row = {a2: max(0, oc[a2] + int(rng.integers(-2, 3))) for a2 in range(A) if rng.random() < 0.6}
                    row = {a2: v for a2, v in row.items() if v}
                    ops.append(("orm", a, c, k, row, ms))
                    oo.append(O.MapUp(O.Dot(a, c), k, O.OrswotRm(O.VClock(dict(row)), ms)))
            else:  # Map Rm
                row = {a2: max(0, clk[a2] + int(rng.integers(-3, 3))) for a2 in range(A) if rng.random() < 0.5}
                row = {a2: v for a2, v in row.items() if v}
                ks = sorted(set(int(z) for z in rng.choice(K, size=int(rng.integers(1, 3)), replace=False)))
                ops.append(("rm", row, ks))
                oo.append(O.MapRm(O.VClock(dict(row)), ks))
        streams.append(ops)
        oops.append(oo)
    return streams, oops


@pytest.mark.parametrize("M,A,seed", [(4, 5, 1), (3, 6, 2), (70, 6, 3), (4, 80, 4)])
def test_map_orswot_apply(gpu_ctx, M, A, seed):
    N, K, T, Dcap = 16, 4, 30, 16
    maps = O.map_orswot_objects(N, K, M, A, seed=60 + seed, steps=160, p_vrm=0.4)
    res, kw, off = _states(gpu_ctx, maps, K, M, A)
    exps = [O.map_fold_objects([m]) for m in maps]
    rng = np.random.default_rng(seed)
    streams, oops = _streams(rng, exps, K, M, A, T)
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in exps for e in x.entries.values()) or \
            any(len(x.deferred) > Dcap for x in exps):
        pytest.skip("past the kernel's deferred capacity")
    Kw = (K + 63) // 64
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    if kw:
        keep, hk, hc = res.def_keep.cpu().numpy(), to_host(res.def_keys), to_host(kw["def_clock"])
        for n in range(N):
            for j in range(off[n], off[n + 1]):
                if keep[j]:
                    dcl[n, cnt[n]], dks[n, cnt[n]] = hc[j], hk[j]
                    cnt[n] += 1
    tdc, tdk, tcnt = to_dev(dcl), to_dev(dks), torch.from_numpy(cnt).cuda()
    ops = cg.map.encode_orswot_map_ops(streams, A, "cuda:0")
    status = cg.map.orswot_apply_batch(res, tdc, tdk, tcnt, ops, ctx=gpu_ctx).cpu().numpy()
    c, e, o, m = to_host(res.clock), to_host(res.ec), to_host(res.oc), to_host(res.ent)
    vn, vc, vm = res.vd_n.cpu().numpy(), to_host(res.vd_clock), to_host(res.vd_mem)
    hdc, hdk, hcnt = to_host(tdc), to_host(tdk), tcnt.cpu().numpy()
    nested = mapdef = 0
    for n in range(N):
        assert status[n] == 0, (n, status[n])
        mw = (lambda k, i: vm[n, k, i]) if vm.ndim == 4 else (lambda k, i: vm[n, k, i:i + 1])  # noqa: E731
        vd = {k: [(vc[n, k, i], O.bitmap_members(mw(k, i))) for i in range(int(vn[n, k]))] for k in range(K)}
        dfr = [(hdc[n, i], O.bitmap_members(hdk[n, i])) for i in range(int(hcnt[n]))]
        got = O.dense_to_map_orswot(c[n], e[n], o[n], m[n], vd, dfr)
        exp = exps[n]
        assert got.clock == exp.clock, n
        assert got.entries == exp.entries, n
        assert got.deferred == exp.deferred, n
        nested += sum(len(x.val.deferred) for x in exp.entries.values())
        mapdef += len(exp.deferred)
    assert nested > 0 and mapdef > 0


def test_map_orswot_apply_unapplied_input_deferred(gpu_ctx):
    """As the counter Map's test: Map-level removes in the input never applied to their keys are
    applied by the first Up's full apply_deferred pass, later passes re-forget the Up's key only."""
    N, K, M, A, T, Dcap = 12, 4, 5, 5, 16, 16
    maps = O.map_orswot_objects(N, K, M, A, seed=61, steps=160, p_vrm=0.3)
    exps = [O.map_fold_objects([m]) for m in maps]
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in exps for e in x.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    res, kw, off = _states(gpu_ctx, maps, K, M, A)
    rng = np.random.default_rng(91)
    Kw = (K + 63) // 64
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    if kw:
        keep, hk, hc = res.def_keep.cpu().numpy(), to_host(res.def_keys), to_host(kw["def_clock"])
        for n in range(N):
            for j in range(off[n], off[n + 1]):
                if keep[j]:
                    dcl[n, cnt[n]], dks[n, cnt[n]] = hc[j], hk[j]
                    cnt[n] += 1
    for n, x in enumerate(exps):  # one more remove from the future, not applied to its keys
        row = np.zeros(A, np.uint64)
        row[0], row[1] = x.clock.get(0) + 1, x.clock.get(1) + 1
        ks = set(int(k) for k in rng.choice(K, size=2, replace=False))
        x.deferred[O.VClock({0: int(row[0]), 1: int(row[1])})] = set(ks)
        dcl[n, cnt[n]] = row
        dks[n, cnt[n], 0] = sum(1 << k for k in ks)
        cnt[n] += 1
    streams, oops = _streams(rng, exps, K, M, A, T)
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in exps for e in x.entries.values()) or \
            any(len(x.deferred) > Dcap for x in exps):
        pytest.skip("past the kernel's deferred capacity")
    tdc, tdk, tcnt = to_dev(dcl), to_dev(dks), torch.from_numpy(cnt).cuda()
    ops = cg.map.encode_orswot_map_ops(streams, A, "cuda:0")
    status = cg.map.orswot_apply_batch(res, tdc, tdk, tcnt, ops, ctx=gpu_ctx).cpu().numpy()
    c, e, o, m = to_host(res.clock), to_host(res.ec), to_host(res.oc), to_host(res.ent)
    vn, vc, vm = res.vd_n.cpu().numpy(), to_host(res.vd_clock), to_host(res.vd_mem)
    hdc, hdk, hcnt = to_host(tdc), to_host(tdk), tcnt.cpu().numpy()
    for n in range(N):
        assert status[n] == 0, (n, status[n])
        vd = {k: [(vc[n, k, i], O.bitmap_members(vm[n, k, i:i + 1])) for i in range(int(vn[n, k]))] for k in range(K)}
        dfr = [(hdc[n, i], O.bitmap_members(hdk[n, i])) for i in range(int(hcnt[n]))]
        got = O.dense_to_map_orswot(c[n], e[n], o[n], m[n], vd, dfr)
        assert got.clock == exps[n].clock and got.entries == exps[n].entries and got.deferred == exps[n].deferred, n


def test_map_orswot_apply_offsets_past_the_pools(gpu_ctx):
    """mem_off / key_off claiming more entries than the pools hold: the pools' lengths
    bound them, so the ops are flagged (status bit 1) and skipped instead of read past the buffers."""
    N, K, M, A, Dcap = 3, 4, 5, 5, 4
    maps = O.map_orswot_objects(N, K, M, A, seed=62, steps=40, p_vrm=0.0)
    res, _, _ = _states(gpu_ctx, maps, K, M, A)
    streams = [[("add", 0, 999, 1, 0, 999, [2])], [("rm", {0: 1}, [0])], [("add", 1, 999, 2, 1, 999, [3])]]
    ops = cg.map.encode_orswot_map_ops(streams, A, "cuda:0")
    mo, ko = ops.mem_off.clone(), ops.key_off.clone()
    mo[1:] = 1 << 20    # op 0 (state 0) claims a million members; op 2 starts past the pool too
    ko[2:] = 1 << 20    # op 1 (state 1) claims a million keys
    bad = ops._replace(mem_off=mo, key_off=ko)
    Kw = (K + 63) // 64
    z = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    st = cg.map.orswot_apply_batch(res, z(N, Dcap, A), z(N, Dcap, Kw),
                                   torch.zeros(N, dtype=torch.int32, device="cuda:0"), bad, ctx=gpu_ctx).cpu().numpy()
    torch.cuda.synchronize()
    assert st[0] & 2 and st[1] & 2 and st[2] & 2, st
    with pytest.raises(TypeError):
        cg.map.orswot_apply_batch(res, z(N, Dcap, A), z(N, Dcap, Kw), torch.zeros(N, dtype=torch.int32, device="cuda:0"),
                                  ops._replace(vcounter=ops.vcounter.to(torch.int32)), ctx=gpu_ctx)


def test_map_orswot_apply_long_deferred_list(gpu_ctx):
    """More Map-level deferred removes than the 16 slots the kernel holds in LDS (round 6: the rest of
    Dcap used in place in the caller's slot arrays): Map Rms from the far future on actor 0 (Ups on
    actors 1..), 20+ removes per state at Dcap = 48, equal to the oracle's Map.apply."""
    N, K, M, A, T, Dcap = 10, 4, 6, 5, 60, 48
    maps = O.map_orswot_objects(N, K, M, A, seed=63, steps=120, p_vrm=0.3)
    exps = [O.map_fold_objects([m]) for m in maps]
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in exps for e in x.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    res, kw, off = _states(gpu_ctx, maps, K, M, A)
    rng = np.random.default_rng(17)
    streams, oops = [], []
    for x in exps:
        clk = {a: x.clock.get(a) for a in range(A)}
        ops, oo = [], []
        for i in range(T):
            if rng.random() < 0.55:
                row = {0: clk[0] + 1000 + i}
                ks = sorted(set(int(z) for z in rng.choice(K, size=int(rng.integers(1, 3)), replace=False)))
                ops.append(("rm", row, ks))
                oo.append(O.MapRm(O.VClock(dict(row)), ks))
            else:
                a = int(rng.integers(1, A))
                c = clk[a] + 1
                clk[a] = c
                k = int(rng.integers(K))
                ms = sorted(set(int(z) for z in rng.choice(M, size=int(rng.integers(1, 3)), replace=False)))
                va, vc = int(rng.integers(1, A)), 500 + i
                ops.append(("add", a, c, k, va, vc, ms))
                oo.append(O.MapUp(O.Dot(a, c), k, O.OrswotAdd(O.Dot(va, vc), ms)))
        streams.append(ops)
        oops.append(oo)
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    Kw = (K + 63) // 64
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    if kw:
        keep, hk, hc = res.def_keep.cpu().numpy(), to_host(res.def_keys), to_host(kw["def_clock"])
        for n in range(N):
            for j in range(off[n], off[n + 1]):
                if keep[j]:
                    dcl[n, cnt[n]], dks[n, cnt[n]] = hc[j], hk[j]
                    cnt[n] += 1
    tdc, tdk, tcnt = to_dev(dcl), to_dev(dks), torch.from_numpy(cnt).cuda()
    ops = cg.map.encode_orswot_map_ops(streams, A, "cuda:0")
    status = cg.map.orswot_apply_batch(res, tdc, tdk, tcnt, ops, ctx=gpu_ctx).cpu().numpy()
    c, e, o, m = to_host(res.clock), to_host(res.ec), to_host(res.oc), to_host(res.ent)
    vn, vc, vm = res.vd_n.cpu().numpy(), to_host(res.vd_clock), to_host(res.vd_mem)
    hdc, hdk, hcnt = to_host(tdc), to_host(tdk), tcnt.cpu().numpy()
    longest = 0
    for n in range(N):
        assert status[n] == 0, (n, status[n])
        mw = (lambda k, i: vm[n, k, i]) if vm.ndim == 4 else (lambda k, i: vm[n, k, i:i + 1])  # noqa: E731
        vd = {k: [(vc[n, k, i], O.bitmap_members(mw(k, i))) for i in range(int(vn[n, k]))] for k in range(K)}
        dfr = [(hdc[n, i], O.bitmap_members(hdk[n, i])) for i in range(int(hcnt[n]))]
        got = O.dense_to_map_orswot(c[n], e[n], o[n], m[n], vd, dfr)
        assert got.clock == exps[n].clock and got.entries == exps[n].entries and got.deferred == exps[n].deferred, n
        longest = max(longest, len(exps[n].deferred))
    assert 20 <= longest <= Dcap
