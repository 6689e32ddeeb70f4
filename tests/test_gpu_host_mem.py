"""GPU parity of the host-memory mode (crdt_mem_kind = CRDT_MEM_HOST, csrc/host_stage.hip): the
lattice and LWWReg entry points on HOST arrays, streamed through the device in chunks, against
the oracle folds (vclock.rs:130-136, pncounter.rs:70-75, gset.rs:38-40, lwwreg.rs:43-45 / :84-98).
Small chunk budgets (tune key stage_kb) force many chunks, group tiles and the chunk-boundary
bookkeeping (accumulation, LWW first-conflict index offsets); pageable and pinned inputs, strided
rows and the refusal paths are covered."""
import ctypes

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import host  # noqa: E402

U64MAX = np.uint64(2**64 - 1)


@pytest.fixture(scope="module")
def hctx():
    c = host.HostContext(0, tune="stage_kb=4")  # 4 KiB chunks: many chunks at test sizes
    yield c
    c.close()


def rand_rows(rng, shape, hi=2**40):
    return rng.integers(0, hi, size=shape, dtype=np.uint64)


@pytest.mark.parametrize("kind", ["vclock", "gcounter", "pncounter", "gset"])
@pytest.mark.parametrize("G,R,W", [(1, 1, 4), (1, 1000, 6), (3, 257, 64), (40, 9, 130), (700, 2, 8)])
def test_lub_many_host(hctx, kind, G, R, W):
    rng = np.random.default_rng(G * 1000 + R + W)
    x = rand_rows(rng, (G, R, W))
    exp = np.bitwise_or.reduce(x, axis=1) if kind == "gset" else x.max(axis=1)
    for g in range(min(G, 3)):  # pin the numpy reduction on a few groups against the oracle
        fold = O.gset_fold(x[g])[0] if kind == "gset" else O.vclock_fold(x[g])[0]
        assert np.array_equal(fold, exp[g])
    got = host.lub_many(kind, x, ctx=hctx)
    assert np.array_equal(got, exp)
    # pinned input, strided rows (a column slice of wider rows), strided output, accumulate
    wide = host.pinned_empty((G, R, W + 3))
    wide[...] = rand_rows(rng, (G, R, W + 3))
    view = wide[:, :, 1:W + 1]
    out_wide = np.zeros((G, W + 5), np.uint64)
    out = out_wide[:, 2:W + 2]
    out[...] = rand_rows(rng, (G, W))
    start = out.copy()
    host.lub_many(kind, view, out=out, accumulate=True, ctx=hctx)
    red = np.bitwise_or.reduce(view, axis=1) if kind == "gset" else view.max(axis=1)
    assert np.array_equal(out, (start | red) if kind == "gset" else np.maximum(start, red))
    assert not out_wide[:, :2].any() and not out_wide[:, W + 2:].any()


def test_lub_many_host_edges(hctx):
    out = np.full((2, 4), 7, np.uint64)
    host.lub_many("vclock", np.zeros((2, 0, 4), np.uint64), out=out, ctx=hctx)
    assert not out.any()  # fold of nothing = VClock::new()
    out[...] = 5
    host.lub_many("vclock", np.zeros((2, 0, 4), np.uint64), out=out, accumulate=True, ctx=hctx)
    assert (out == 5).all()
    big = host.HostContext(0)  # default 256 MiB chunks: one chunk
    x = rand_rows(np.random.default_rng(3), (5000, 256))
    assert np.array_equal(host.lub_many("gcounter", x, ctx=big), x.max(axis=0))
    big.close()


@pytest.mark.parametrize("kind", ["vclock", "pncounter", "gset"])
@pytest.mark.parametrize("N,W", [(1, 4), (1000, 6), (37, 300)])
def test_merge_batch_host(hctx, kind, N, W):
    rng = np.random.default_rng(N + W)
    a, b = rand_rows(rng, (N, W)), rand_rows(rng, (N, W))
    exp = (a | b) if kind == "gset" else np.maximum(a, b)
    if kind == "vclock":
        assert np.array_equal(O.vclock_merge_pairs(a, b), exp)
    got = host.merge_batch(kind, a.copy(), b, ctx=hctx)
    assert np.array_equal(got, exp)
    # strided self / other rows
    sw, ow = rand_rows(rng, (N, W + 2)), rand_rows(rng, (N, W + 1))
    s0 = sw.copy()
    host.merge_batch(kind, sw[:, 1:W + 1], ow[:, :W], ctx=hctx)
    e2 = (s0[:, 1:W + 1] | ow[:, :W]) if kind == "gset" else np.maximum(s0[:, 1:W + 1], ow[:, :W])
    assert np.array_equal(sw[:, 1:W + 1], e2)
    assert np.array_equal(sw[:, 0], s0[:, 0]) and np.array_equal(sw[:, W + 1], s0[:, W + 1])


def lww_case(rng, G, R, n_markers):
    m = rng.integers(0, n_markers, size=(G, R), dtype=np.uint64)
    v = rng.integers(0, 3, size=(G, R), dtype=np.uint64)
    return m, v


@pytest.mark.parametrize("G,R,nm", [(1, 5000, 50), (7, 1300, 4000), (300, 3, 2), (1, 1, 5), (2000, 17, 5)])
def test_lwwreg_lub_many_host(hctx, G, R, nm):
    rng = np.random.default_rng(G + R)
    m, v = lww_case(rng, G, R, nm)
    got = host.lwwreg_lub_many(m, v, ctx=hctx)
    for g in range(G):
        om, ov, fc, _ = O.lwwreg_fold(m[g], v[g])
        assert (int(got.marker[g]), int(got.val[g]), int(got.first_conflict[g])) == (om, ov, fc), g


def test_lwwreg_conflict_in_later_chunk(hctx):
    """The first conflicting merge sits beyond the first chunk (4 KiB = 256 replicas per chunk
    at G = 1): its index must be the global one."""
    R = 2000
    m = np.arange(1, R + 1, dtype=np.uint64)
    v = np.zeros(R, np.uint64)
    m[1500] = m[1499]
    v[1500] = 9  # same marker, different value -> Err at replica 1500
    m[1800] = m[1799] = 10**9
    v[1800] = 1  # a later conflict too
    got = host.lwwreg_lub_many(m, v, ctx=hctx)
    om, ov, fc, _ = O.lwwreg_fold(m, v)
    assert fc == 1500 and int(got.first_conflict[0]) == 1500
    assert (int(got.marker[0]), int(got.val[0])) == (om, ov)


def test_lwwreg_merge_batch_host(hctx):
    rng = np.random.default_rng(5)
    N = 3000
    sm, sv = lww_case(rng, 1, N, 4)
    om_, ov_ = lww_case(rng, 1, N, 4)
    sm, sv, om_, ov_ = sm[0].copy(), sv[0].copy(), om_[0], ov_[0]
    s0m, s0v = sm.copy(), sv.copy()
    conflict = host.lwwreg_merge_batch(sm, sv, om_, ov_, ctx=hctx)
    for i in range(N):
        em, ev, fc, _ = O.lwwreg_fold(np.array([s0m[i], om_[i]]), np.array([s0v[i], ov_[i]]))
        assert (int(sm[i]), int(sv[i]), int(conflict[i])) == (em, ev, int(fc == 1)), i


def test_host_mode_refusals(hctx):
    # a device pointer handed to host mode is rejected, not read
    d = torch.zeros((4, 8), dtype=torch.int64, device="cuda")
    out = np.zeros(8, np.uint64)
    rc = hctx.raw("crdt_vclock_lub_many", ctypes.c_void_p(d.data_ptr()), 1, 4, 8, 8, 32, ctypes.c_void_p(out.ctypes.data), 8, 0)
    assert rc == cg._abi.CRDT_EINVAL
    # entry points without a host path refuse the mode
    assert hctx.raw("crdt_vclock_apply_batch", None, 0, 0, 0, None, None, None, 0, None) == -4
    assert hctx.raw("crdt_orswot_lub_many", None, None) == cg._abi.CRDT_EINVAL  # host-capable: NULL batch
    assert hctx.raw("crdt_map_lub_many", None, None) == cg._abi.CRDT_EINVAL  # host-capable too
    assert hctx.raw("crdt_map_apply_batch", None, None, None, None, 0, None, None) == -4
    assert hctx.raw("crdt_vclock_ingest", None, None, 0, None, 0, None, 0, None) == -4
    # (sharded entry points check for a communicator first: none on this ctx)
    assert hctx.raw("crdt_vclock_lub_many_sharded", None, 0, 0, 0, 0, 0, None) == cg._abi.CRDT_EINVAL
    assert hctx.lib.crdt_ctx_mem_kind(hctx.ptr) == cg._abi.CRDT_MEM_HOST
    # device mode is unaffected on another ctx
    ctx = cg.Context(0)
    assert ctx.lib.crdt_ctx_mem_kind(ctx.ptr) == cg._abi.CRDT_MEM_DEVICE


def test_orswot_host_lub_many(hctx):
    """crdt_orswot_lub_many on host arrays == the device-pointer call == the oracle fold."""
    c, e, off, dcl, dmem = O.gen_orswot(7, 50, 70, 9, kmax=12, p_def=0.4)
    D = int(off[-1])
    got = host.orswot_lub_many(c, e, def_off=[0, D], def_clock=dcl, def_members=dmem, ctx=hctx)
    dev = cg.orswot.lub_many(torch.from_numpy(c.view(np.int64)).cuda(), torch.from_numpy(e.view(np.int64)).cuda(),
                             def_off=[0, D], def_clock=torch.from_numpy(dcl.view(np.int64)).cuda(),
                             def_members=torch.from_numpy(dmem.view(np.int64)).cuda())
    np.testing.assert_array_equal(got.clock, dev.clock.cpu().numpy().view(np.uint64))
    np.testing.assert_array_equal(got.entries, dev.entries.cpu().numpy().view(np.uint64))
    oc, oe, odef, _ = O.orswot_fold(c, e, off, dcl, dmem)
    np.testing.assert_array_equal(got.clock, oc)
    np.testing.assert_array_equal(got.entries, oe)
    surv = {(tuple(int(x) for x in dcl[d]), O.bitmap_members(got.def_members[d])) for d in range(D) if got.def_keep[d]}
    assert D > 0 and surv == odef


@pytest.mark.parametrize("stage_kb,G,R", [(24, 1, 50), (40, 3, 37), (12, 2, 5), (1 << 18, 1, 50)])
def test_orswot_host_lub_many_streamed(stage_kb, G, R):
    """Replica chunks streamed through the stage buffers (running join in slot 0, deferred removes
    settled once at the end) == the whole-batch staging == the oracle fold, per group; chunk sizes
    from 1 to all replicas of a group."""
    M, A = 70, 9
    rng = np.random.default_rng(stage_kb + G)
    cs, es, offs, roffs, dcls, dmems = [], [], [0], [], [], []
    for g in range(G):
        c, e, off, dcl, dmem = O.gen_orswot(int(rng.integers(1 << 30)), R, M, A, kmax=12, p_def=0.4)
        roffs.append(off)  # per-replica offsets (the oracle's form); the library takes per-group ones
        cs.append(c)
        es.append(e)
        offs.append(offs[-1] + int(off[-1]))
        dcls.append(dcl)
        dmems.append(dmem)
    c, e = np.stack(cs), np.stack(es)
    dcl, dmem = np.concatenate(dcls), np.concatenate(dmems)
    res = []
    for hs in (1, 0):
        ctx = host.HostContext(0, tune=f"stage_kb={stage_kb},hstream={hs}")
        res.append(host.orswot_lub_many(c, e, def_off=offs, def_clock=dcl, def_members=dmem, ctx=ctx))
        ctx.close()
    for x in ("clock", "entries", "def_keep", "def_members"):
        np.testing.assert_array_equal(getattr(res[0], x), getattr(res[1], x), err_msg=x)
    for g in range(G):
        oc, oe, odef, _ = O.orswot_fold(cs[g], es[g], roffs[g], dcls[g], dmems[g])
        np.testing.assert_array_equal(res[0].clock[g], oc)
        np.testing.assert_array_equal(res[0].entries[g], oe)
        surv = {(tuple(int(x) for x in dcl[d]), O.bitmap_members(res[0].def_members[d]))
                for d in range(offs[g], offs[g + 1]) if res[0].def_keep[d]}
        assert surv == odef


def test_orswot_host_merge_batch(hctx):
    from orswot_apply_util import dense_states, oracle_streams, replay_streams, to_object
    N, M, n_origins = 30, 40, 4
    streams = replay_streams(5, 2 * N, n_origins, M, 200)
    states = oracle_streams([O.Orswot() for _ in streams], streams)
    lhs, rhs = states[:N], states[N:]
    Dcap = max(1, max(len(a.deferred) + len(b.deferred) for a, b in zip(lhs, rhs)))
    me = [np.ascontiguousarray(x) for x in dense_states(lhs, M, n_origins, Dcap)]
    other = [np.ascontiguousarray(x) for x in dense_states(rhs, M, n_origins, Dcap)]
    me[4], other[4] = me[4].astype(np.uint32), other[4].astype(np.uint32)
    status = host.orswot_merge_batch(tuple(me), tuple(other), ctx=hctx)
    assert (status == 0).all(), status
    for i, (a, b) in enumerate(zip(lhs, rhs)):
        exp = a.copy()
        exp.merge(b.copy())
        assert to_object(me[0], me[1], me[2], me[3], me[4], i) == exp, i
    assert sum(len(s.deferred) for s in lhs) > 0


def test_map_host_lub_many(hctx):
    """crdt_map_lub_many on host arrays == the device-pointer call (bit for bit, every output)."""
    dfr = O.synth_map_deferred(0x5EED0044, 300, 40, 8, 30, p_def=0.3)
    rows, dcl, dks = dfr
    d = O.synth_map(0x5EED0044, 300, 40, 8, 2, 30, keys=np.arange(40), deferred=dfr)
    D = rows.shape[0]
    got = host.map_lub_many(d["clock"], d["ec"], d["vclk"], d["vval"], def_off=[0, D], def_row=rows, def_clock=dcl,
                            def_keys=dks, ctx=hctx)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64)).cuda()  # noqa: E731
    dev = cg.map.lub_many(t(d["clock"]), t(d["ec"]), t(d["vclk"]), t(d["vval"]), def_off=[0, D],
                          def_row=torch.from_numpy(rows.astype(np.int32)).cuda(), def_clock=t(dcl), def_keys=t(dks),
                          vout=4, check=False)
    h = lambda x: x.cpu().numpy().view(np.uint64) if x.dtype == torch.int64 else x.cpu().numpy()  # noqa: E731
    np.testing.assert_array_equal(got.clock[0], h(dev.clock))
    np.testing.assert_array_equal(got.ec[0], h(dev.ec))
    np.testing.assert_array_equal(got.vclk[0], h(dev.vclk))
    np.testing.assert_array_equal(got.vval[0], h(dev.vval))
    np.testing.assert_array_equal(got.def_keep, h(dev.def_keep).astype(np.uint8))
    assert D > 0 and got.ec.any()


@pytest.mark.parametrize("stage_kb,vout,src", [(64, 4, "synth"), (24, 2, "replay"), (40, 4, "replay"),
                                               (1 << 18, 4, "synth"), (16, 8, "synth")])
def test_map_host_lub_many_streamed(stage_kb, vout, src):
    """Replica chunks streamed with the running fold as replica 0 (its surviving removes carried)
    == whole-batch staging, every output word, == the oracle fold; vout 2 (no widening; keys
    needing more slots restart with 8), 4 (V = 2 inputs widened to 4 slots) and 8."""
    if src == "synth":
        dfr = O.synth_map_deferred(0x5EED0045, 200, 40, 8, 30, p_def=0.3)
        rows, dcl, dks = dfr
        d = O.synth_map(0x5EED0045, 200, 40, 8, 2, 30, keys=np.arange(40), deferred=dfr)
    else:
        maps = O.gen_map_replicas(11 + stage_kb, 60, 12, 5, steps=400, p_rm=0.3, p_up=0.4)
        d = O.map_to_dense(maps, 12, 5, max(1, O.max_vals(maps)))
        rows, dcl, dks = d["def_row"], d["def_clock"], d["def_keys"]
    D = rows.shape[0]
    res = []
    for hs in (1, 0):
        ctx = host.HostContext(0, tune=f"stage_kb={stage_kb},hstream={hs}")
        res.append(host.map_lub_many(d["clock"], d["ec"], d["vclk"], d["vval"], def_off=[0, D], def_row=rows,
                                     def_clock=dcl, def_keys=dks, vout=vout, ctx=ctx))
        ctx.close()
    for f in res[0]._fields:
        np.testing.assert_array_equal(getattr(res[0], f), getattr(res[1], f), err_msg=f)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], rows, dcl, dks, vout)
    if int(res[0].flags[0]) & 1:  # more values than vout on some key: reported alike by both forms
        assert int(exp[4].max()) > vout
        return
    np.testing.assert_array_equal(res[0].clock[0], exp[0])
    np.testing.assert_array_equal(res[0].ec[0], exp[1])
    np.testing.assert_array_equal(res[0].vclk[0], exp[2])
    np.testing.assert_array_equal(res[0].vval[0], exp[3])
    np.testing.assert_array_equal(res[0].nval[0], exp[4])
    got = {(tuple(int(x) for x in dcl[j]), O.bitmap_members(res[0].def_keys[j])) for j in np.flatnonzero(res[0].def_keep)}
    assert got == exp[5]


@pytest.mark.parametrize("hs", [1, 0])
def test_map_host_def_row_past_r(hs):
    """A remove whose def_row == R (held by no replica): the streamed and the whole-batch host forms
    both report flags bit 1, as the device fold does (the streamed form used to drop it)."""
    dfr = O.synth_map_deferred(0x5EED0046, 100, 20, 8, 6, p_def=0.3)
    rows, dcl, dks = dfr
    d = O.synth_map(0x5EED0046, 100, 20, 8, 2, 6, keys=np.arange(20), deferred=dfr)
    rows = rows.copy()
    rows[-1] = 100
    D = rows.shape[0]
    ctx = host.HostContext(0, tune=f"stage_kb=64,hstream={hs}")
    res = host.map_lub_many(d["clock"], d["ec"], d["vclk"], d["vval"], def_off=[0, D], def_row=rows,
                            def_clock=dcl, def_keys=dks, vout=4, ctx=ctx)
    ctx.close()
    assert D > 1 and int(res.flags[0]) & 2


def test_map_host_merge_batch(hctx):
    from test_gpu_merge_batch import replay_maps
    N, K, n_origins = 20, 10, 4
    maps = replay_maps(9, 2 * N, n_origins, K, 150)
    lhs, rhs = maps[:N], maps[N:]
    exp = []
    for a, b in zip(lhs, rhs):
        x = a.copy()
        x.merge(b.copy())
        exp.append(x)
    V = max(1, O.max_vals(exp), O.max_vals(lhs), O.max_vals(rhs))
    Dcap = max(1, max(len(m.deferred) for m in list(lhs) + list(rhs) + exp))

    def side(ms):
        dd = O.map_to_dense(ms, K, n_origins, V)
        Kw = (K + 63) // 64
        dcl = np.zeros((N, Dcap, n_origins), np.uint64)
        dks = np.zeros((N, Dcap, Kw), np.uint64)
        cnt = np.zeros(N, np.uint32)
        for j, r in enumerate(dd["def_row"].astype(np.int64)):
            dcl[r, cnt[r]] = dd["def_clock"][j]
            dks[r, cnt[r]] = dd["def_keys"][j]
            cnt[r] += 1
        return tuple(np.ascontiguousarray(x) for x in (dd["clock"], dd["ec"], dd["vclk"], dd["vval"], dcl, dks, cnt))

    me, other = side(lhs), side(rhs)
    status = host.map_merge_batch(me, other, ctx=hctx)
    assert (status == 0).all(), status
    for i, e in enumerate(exp):
        deferred = [(me[4][i, j], O.bitmap_members(me[5][i, j])) for j in range(int(me[6][i]))]
        got = O.dense_to_map(me[0][i], me[1][i], me[2][i], me[3][i], deferred)
        assert got == e, i


# ---- the value-typed Maps in host mode (round 5: whole-batch staging) -----------------------------
def _host_deferred(out, dcl):
    return {(tuple(int(x) for x in dcl[d]), O.bitmap_members(out["def_keys"][d]))
            for d in np.flatnonzero(out["def_keep"])}


@pytest.mark.parametrize("W", [1, 2])
def test_map_counter_host_lub_many(hctx, W):
    """crdt_map_counter_lub_many from host arrays equals the oracle's left fold (map.rs:140-220 with
    the counters' merge / forget); the chunk-skip path (A = 32) and the generic one (A = 5)."""
    for A, seed in ((32, 3), (5, 4)):
        maps = O.map_counter_objects(40, 6, A, W, seed=seed, steps=240, p_rm=0.3)
        exp = O.map_fold_objects(maps)
        d = O.map_counter_to_dense(maps, 6, A, W)
        D = d["def_row"].shape[0]
        out = host.map_counter_lub_many(d["clock"], d["ec"], d["val"], def_off=[0, D] if D else None,
                                        def_row=d["def_row"], def_clock=d["def_clock"], def_keys=d["def_keys"], ctx=hctx)
        assert int(out["flags"][0]) == 0
        dset = _host_deferred(out, d["def_clock"]) if D else set()
        got = O.dense_to_map_counter(out["clock"][0], out["ec"][0], out["val"][0],
                                     [(np.array(rm, np.uint64), ks) for rm, ks in dset])
        assert got == exp


@pytest.mark.parametrize("M,A", [(6, 4), (70, 80)])
def test_map_orswot_host_lub_many(hctx, M, A):
    """(M = 70, A = 80: the wide kernel with two-word member masks, from host memory.)"""
    maps = O.map_orswot_objects(30, 4, M, A, seed=5, steps=200, p_vrm=0.5)
    exp = O.map_fold_objects(maps)
    d = O.map_orswot_to_dense(maps, 4, M, A)
    D, Dv = d["def_row"].shape[0], d["vd_clock"].shape[0]
    out = host.map_orswot_lub_many(d["clock"], d["ec"], d["oc"], d["ent"], d["vd_off"],
                                   d["vd_clock"] if Dv else None, d["vd_members"] if Dv else None,
                                   def_off=[0, D] if D else None, def_row=d["def_row"], def_clock=d["def_clock"],
                                   def_keys=d["def_keys"], ctx=hctx)
    assert int(out["flags"][0]) == 0
    dset = _host_deferred(out, d["def_clock"]) if D else set()
    vm = out["vd_mem"]
    mw = (lambda k, i: vm[0, k, i]) if vm.ndim == 4 else (lambda k, i: vm[0, k, i:i + 1])  # noqa: E731
    vd = {k: [(out["vd_clock"][0, k, i], O.bitmap_members(mw(k, i)))
              for i in range(int(out["vd_n"][0, k]))] for k in range(4)}
    got = O.dense_to_map_orswot(out["clock"][0], out["ec"][0], out["oc"][0], out["ent"][0], vd,
                                [(np.array(rm, np.uint64), ks) for rm, ks in dset])
    assert got == exp


def test_map_nested_host_lub_many(hctx):
    maps = O.nested_map_objects(30, 3, 5, 4, seed=6, steps=240, p_irm=0.5, p_ooo=0.8, p_rm=0.3)
    exp = O.map_fold_objects(maps)
    V = max([len(ie.val.vals) for m in maps for e in m.entries.values() for ie in e.val.entries.values()] + [1])
    d = O.nested_map_to_dense(maps, 3, 5, 4, V)
    D, Di = d["def_row"].shape[0], d["id_clock"].shape[0]
    out = host.map_nested_lub_many(d["clock"], d["ec"], d["ic"], d["iec"], d["ivc"], d["ivv"], d["id_off"],
                                   d["id_clock"] if Di else None, d["id_keys"] if Di else None,
                                   def_off=[0, D] if D else None, def_row=d["def_row"], def_clock=d["def_clock"],
                                   def_keys=d["def_keys"], ctx=hctx)
    assert int(out["flags"][0]) == 0
    dset = _host_deferred(out, d["def_clock"]) if D else set()
    idef = {k: [(out["id_clock"][0, k, i], O.bitmap_members(out["id_keys"][0, k, i:i + 1]))
                for i in range(int(out["id_n"][0, k]))] for k in range(3)}
    got = O.dense_to_nested_map(out["clock"][0], out["ec"][0], out["ic"][0], out["iec"][0], out["ivc"][0],
                                out["ivv"][0], out["nval"][0], idef, [(np.array(rm, np.uint64), ks) for rm, ks in dset])
    from test_gpu_map_nested import canon
    assert canon(got) == canon(exp)


def test_map_value_host_lub_many_deep(hctx):
    """Host memory (round 6): a Map<K, Orswot> fold with keys past 16 nested removes (Vd = 64) and a
    nested Map fold with keys past 16 inner removes and K2 = 100 inner keys (Id = 64, two mask words):
    the staged deep passes, equal to the oracle."""
    from test_gpu_map_nested import canon
    from test_gpu_map_nested_deep import _deep_nested
    from test_gpu_map_orswot_deep import _deep_maps
    rng = np.random.default_rng(31)
    R, K, M, A = 8, 3, 5, 8
    maps = _deep_maps(rng, R, K, M, A)
    exp = O.map_fold_objects(maps)
    assert max(len(e.val.deferred) for e in exp.entries.values()) > 16
    d = O.map_orswot_to_dense(maps, K, M, A)
    out = host.map_orswot_lub_many(d["clock"], d["ec"], d["oc"], d["ent"], d["vd_off"], d["vd_clock"],
                                   d["vd_members"], ctx=hctx, vd_cap=64)
    assert int(out["flags"][0]) == 0
    vd = {k: [(out["vd_clock"][0, k, i], O.bitmap_members(out["vd_mem"][0, k, i:i + 1]))
              for i in range(int(out["vd_n"][0, k]))] for k in range(K)}
    got = O.dense_to_map_orswot(out["clock"][0], out["ec"][0], out["oc"][0], out["ent"][0], vd, [])
    assert got == exp
    K2 = 100
    maps = _deep_nested(rng, 6, 2, K2, 8)
    exp = O.map_fold_objects(maps)
    assert max(len(e.val.deferred) for e in exp.entries.values()) > 16
    d = O.nested_map_to_dense(maps, 2, K2, 8, 8)
    out = host.map_nested_lub_many(d["clock"], d["ec"], d["ic"], d["iec"], d["ivc"], d["ivv"], d["id_off"],
                                   d["id_clock"], d["id_keys"], ctx=hctx, id_cap=64)
    assert int(out["flags"][0]) == 0 and out["id_keys"].shape == (1, 2, 64, 2)
    idef = {k: [(out["id_clock"][0, k, i], O.bitmap_members(out["id_keys"][0, k, i]))
                for i in range(int(out["id_n"][0, k]))] for k in range(2)}
    got = O.dense_to_nested_map(out["clock"][0], out["ec"][0], out["ic"][0], out["iec"][0], out["ivc"][0],
                                out["ivv"][0], out["nval"][0], idef, [])
    assert canon(got) == canon(exp)


def test_map_value_host_lub_many_empty_batch(hctx):
    """R == 0 from host memory with a NULL vd_off / id_off, as the device path accepts:
    the empty fold Map::new(), no copy from NULL."""
    z = lambda *s: np.zeros(s, np.uint64)  # noqa: E731
    K, M, A, K2, V = 3, 5, 4, 2, 2
    out = host.map_orswot_lub_many(z(0, A), z(0, K, A), z(0, K, A), z(0, K, M, A), None, ctx=hctx)
    assert int(out["flags"][0]) == 0 and not out["clock"].any() and not out["ec"].any() and not out["vd_n"].any()
    out = host.map_nested_lub_many(z(0, A), z(0, K, A), z(0, K, A), z(0, K, K2, A), z(0, K, K2, V, A),
                                   z(0, K, K2, V), None, ctx=hctx)
    assert int(out["flags"][0]) == 0 and not out["clock"].any() and not out["nval"].any()
