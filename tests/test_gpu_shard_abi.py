"""GPU: the C ABI's own RCCL sharded lub (crdt_*_lub_many_sharded, crdt_orswot_lub_many_sharded)
at world size 1 on one MI355X — the communicator setup, the exchange calls and the re-merge
bookkeeping (deferred pooling by group, survivor compaction) run for real; the multi-rank data
movement is the torch.distributed twin's, which tests/test_dist_cpu.py covers under gloo."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host, umax_torch

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


@pytest.fixture(scope="module")
def comm_ctx():
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    cg.shard.comm_init(ctx, cg.shard.unique_id(), 1, 0)
    assert cg.shard.comm_info(ctx) == (1, 0)
    yield ctx
    cg.shard.comm_destroy(ctx)
    assert cg.shard.comm_info(ctx) == (0, -1)
    ctx.close()


def test_sharded_needs_comm(gpu_ctx):
    x = torch.zeros((4, 8), dtype=torch.int64, device="cuda:0")
    with pytest.raises(cg.CrdtGpuError):
        cg.shard.lub_many_sharded("vclock", x, ctx=cg.Context(0))


@pytest.mark.parametrize("kind,W", [("vclock", 64), ("gcounter", 256), ("pncounter", 2 * 33), ("gset", 17)])
@pytest.mark.parametrize("G,R", [(1, 1000), (3, 77), (2, 0)])
def test_lattice_sharded_world1(comm_ctx, kind, W, G, R):
    rows = O.synth_matrix(0x5EED0011 + W, G * R, W, 1 if kind == "gset" else 0).reshape(G, R, W)
    x = to_dev(rows)
    got = to_host(cg.shard.lub_many_sharded(kind, x, ctx=comm_ctx))
    if R == 0:
        exp = np.zeros((G, W), np.uint64)
    elif kind == "gset":
        exp = np.bitwise_or.reduce(rows, axis=1)
    else:
        exp = to_host(umax_torch(x, 1))
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("devoff", [False, True])
@pytest.mark.parametrize("seed,G,R,M,A", [(1, 1, 40, 64, 8), (2, 3, 12, 50, 8), (3, 2, 1, 130, 65)])
def test_orswot_sharded_world1(comm_ctx, seed, G, R, M, A, devoff):
    """devoff: the deferred offsets as a device tensor (crdt_orswot_lub_many_sharded_doff)."""
    parts = [O.gen_orswot(seed * 10 + g, R, M, A, kmax=10, p_def=0.4) for g in range(G)]
    clock = np.stack([p[0] for p in parts])
    entries = np.stack([p[1] for p in parts])
    off = [0]
    for p in parts:
        off.append(off[-1] + p[3].shape[0])
    Mw = (M + 63) // 64
    dcl = np.concatenate([p[3] for p in parts]).reshape(-1, A)
    dmem = np.concatenate([p[4] for p in parts]).reshape(-1, Mw)
    kw = dict(def_off=off, def_clock=to_dev(dcl), def_members=to_dev(dmem)) if off[-1] else {}
    if devoff:
        kw["def_off"] = torch.tensor(off, dtype=torch.int64, device="cuda:0")
    res = cg.shard.orswot_lub_many_sharded(to_dev(clock), to_dev(entries), ctx=comm_ctx, **kw)
    got_c, got_e = to_host(res.clock), to_host(res.entries)
    got_d = cg.shard.deferred_groups(res, G)
    for g, (c, e, o, d, m) in enumerate(parts):
        oc, oe, odef, _ = O.orswot_fold(c, e, o, d, m)
        np.testing.assert_array_equal(got_c[g], oc)
        np.testing.assert_array_equal(got_e[g], oe)
        assert got_d[g] == odef, g
    # a too-small def_cap is retried with exactly enough room
    small = cg.shard.orswot_lub_many_sharded(to_dev(clock), to_dev(entries), ctx=comm_ctx, def_cap=1, **kw)
    assert cg.shard.deferred_groups(small, G) == got_d


@pytest.mark.parametrize("bad", [[1, 3, 5], [0, 4, 3], [0, 2, 4]])
def test_orswot_sharded_doff_invalid(comm_ctx, bad):
    """Invalid device offsets (entry 0 != 0, decreasing, entry G != D) are refused after the count
    exchange (EINVAL on the rank that passed them), not read out of range; the ctx stays usable."""
    G, R, M, A = 2, 6, 40, 5
    parts = [O.gen_orswot(70 + g, R, M, A, kmax=6, p_def=0.5) for g in range(G)]
    clock = to_dev(np.stack([p[0] for p in parts]))
    entries = to_dev(np.stack([p[1] for p in parts]))
    D = 5
    dcl = torch.zeros((D, A), dtype=torch.int64, device="cuda:0")
    dmb = torch.zeros((D, 1), dtype=torch.int64, device="cuda:0")
    with pytest.raises(cg.CrdtGpuError, match="def_off"):
        cg.shard.orswot_lub_many_sharded(clock, entries, torch.tensor(bad, dtype=torch.int64, device="cuda:0"),
                                         dcl, dmb, ctx=comm_ctx)
    ok = cg.shard.orswot_lub_many_sharded(clock, entries, ctx=comm_ctx)
    for g, (c, e, _, _, _) in enumerate(parts):
        np.testing.assert_array_equal(to_host(ok.clock[g]), O.orswot_fold(c, e)[0])


@pytest.mark.parametrize("G,R,base", [(3, 201, 0), (2, 57, 1000), (1, 0, 7)])
def test_lwwreg_sharded_world1(comm_ctx, G, R, base):
    """crdt_lwwreg_lub_many_sharded at world 1: the global fold is the local one, conflicts are
    reported at base + local index (lwwreg.rs:84-98)."""
    m = O.synth_matrix(47, G, max(R, 1), 2)[:, :R] % np.uint64(7)
    v = O.synth_matrix(47, G, max(R, 1), 3)[:, :R] % np.uint64(2)
    fm, fv, fc = cg.shard.lwwreg_lub_many_sharded(to_dev(m), to_dev(v), base, ctx=comm_ctx)
    fm, fv, fc = to_host(fm), to_host(fv), to_host(fc)
    for g in range(G):
        if R == 0:
            assert int(fc[g]) == 2**64 - 1
            continue
        om, ov, of, _ = O.lwwreg_fold(m[g], v[g])
        assert (int(fm[g]), int(fv[g])) == (om, ov)
        assert int(fc[g]) == (of if of == 2**64 - 1 else of + base)
    assert R == 0 or any(int(x) != 2**64 - 1 for x in fc)


@pytest.mark.parametrize("devoff", [False, True])
@pytest.mark.parametrize("k0,Kk", [(0, 29), (5, 15), (20, 9), (3, 0)])
def test_map_sharded_world1(comm_ctx, k0, Kk, devoff):
    """crdt_map_lub_many_sharded at world 1 over a key range: the rank's keys equal the oracle's
    whole-map fold restricted to them, and the surviving removes' key sets (over ALL keys) hold
    exactly this rank's keys of them (the bitmap restriction / placement around the exchange)."""
    import dist_world2_data as D
    d = D.map_input()
    K = d["ec"].shape[1]
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"], 8)
    Dn = d["def_row"].shape[0]
    t = lambda a: to_dev(np.ascontiguousarray(a))  # noqa: E731
    off = torch.tensor([0, Dn], dtype=torch.int64, device="cuda:0") if devoff else [0, Dn]
    res = cg.shard.map_lub_many_sharded(t(d["clock"]), t(d["ec"][:, k0:k0 + Kk]), t(d["vclk"][:, k0:k0 + Kk]),
                                        t(d["vval"][:, k0:k0 + Kk]), k0, K, def_off=off,
                                        def_row=torch.from_numpy(d["def_row"].astype(np.int32)).cuda(),
                                        def_clock=t(d["def_clock"]), def_keys=t(d["def_keys"]), vout=8, ctx=comm_ctx)
    np.testing.assert_array_equal(to_host(res.clock), exp[0])
    np.testing.assert_array_equal(to_host(res.ec), exp[1][k0:k0 + Kk])
    np.testing.assert_array_equal(to_host(res.vclk), exp[2][k0:k0 + Kk])
    np.testing.assert_array_equal(to_host(res.vval), exp[3][k0:k0 + Kk])
    got = cg.map.deferred_set(t(d["def_clock"]), res.def_keep, res.def_keys)
    want = {(c, frozenset(k for k in ks if k0 <= k < k0 + Kk)) for c, ks in exp[5]}
    if Kk:
        assert got == want and len(want) > 0
    else:  # an empty key shard: the clock lub and the removes' survival alone
        assert {c for c, _ in got} == {c for c, _ in want} and len(want) > 0


def test_config5_shard_world1(comm_ctx):
    """Config 5 at full per-GPU size through crdt_vclock_lub_many_sharded over the ctx's RCCL
    communicator: 1,048,576 VClock replicas x 1,024 actors (8 GiB) — sampled
    actor columns against the oracle's fold, every column against a torch unsigned max of the same
    HBM rows, and against the unsharded lub_many."""
    from dist_world2_data import C5_A, C5_COLS, C5_R, C5_SEED, c5_expected_columns
    x = torch.empty((C5_R, C5_A), dtype=torch.int64, device="cuda:0")
    cg.synth_fill(comm_ctx, x, C5_SEED, 0, first_row=0)
    got = to_host(cg.shard.lub_many_sharded("vclock", x, ctx=comm_ctx))
    np.testing.assert_array_equal(got[C5_COLS], c5_expected_columns(C5_R))
    np.testing.assert_array_equal(got, to_host(umax_torch(x, 0)))
    np.testing.assert_array_equal(got, to_host(cg.vclock.lub_many(x, ctx=comm_ctx)))
    assert (got != 0).all()
    del x
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k0,Kk", [(0, 29), (5, 15), (20, 9), (3, 0)])
def test_value_maps_sharded_world1(comm_ctx, k0, Kk):
    """The value-typed Maps' key-sharded folds (round 5) at world 1 over a key range: the rank's keys
    equal the unsharded fold of every key restricted to them (itself parity-tested against the
    oracle), and the surviving removes' key sets hold exactly this rank's keys of the unsharded ones."""
    import dist_world2_data as D
    d = D.map_input()
    K = d["ec"].shape[1]
    R = d["clock"].shape[0]
    Dn = d["def_row"].shape[0]
    t = lambda a: to_dev(np.ascontiguousarray(a))  # noqa: E731
    kw = dict(def_off=[0, Dn], def_row=torch.from_numpy(d["def_row"].astype(np.int32)).cuda(),
              def_clock=t(d["def_clock"]), def_keys=t(d["def_keys"]))
    mask = np.zeros(((K + 63) // 64,), np.uint64)
    for k in range(k0, k0 + Kk):
        mask[k // 64] |= np.uint64(1) << np.uint64(k % 64)
    vc = d["vclk"]
    if vc.shape[2] < 2:
        vc = np.concatenate([vc, np.zeros(vc.shape[:2] + (2 - vc.shape[2],) + vc.shape[3:], np.uint64)], axis=2)

    def same(full, sh, rows):
        np.testing.assert_array_equal(to_host(sh.clock), to_host(full.clock))
        for nm in rows:
            np.testing.assert_array_equal(to_host(getattr(sh, nm)), to_host(getattr(full, nm))[k0:k0 + Kk], err_msg=nm)
        np.testing.assert_array_equal(sh.def_keep.cpu().numpy(), full.def_keep.cpu().numpy())
        np.testing.assert_array_equal(to_host(sh.def_keys), to_host(full.def_keys) & mask[None])
        assert full.def_keep.cpu().numpy().any()

    for W in (1, 2):
        val = np.ascontiguousarray(vc[:, :, :W])
        full = cg.map.counter_lub_many(t(d["clock"]), t(d["ec"]), t(val), ctx=comm_ctx, **kw)
        sh = cg.shard.map_counter_lub_many_sharded(t(d["clock"]), t(d["ec"][:, k0:k0 + Kk]), t(val[:, k0:k0 + Kk]),
                                                   k0, K, ctx=comm_ctx, **kw)
        same(full, sh, ("ec", "val"))
    oc, ent = np.ascontiguousarray(d["ec"]), np.ascontiguousarray(vc[:, :, :2])
    full = cg.map.orswot_lub_many(t(d["clock"]), t(d["ec"]), t(oc), t(ent),
                                  torch.zeros(R * K + 1, dtype=torch.int64, device="cuda:0"), ctx=comm_ctx, **kw)
    sh = cg.shard.map_orswot_lub_many_sharded(t(d["clock"]), t(d["ec"][:, k0:k0 + Kk]), t(oc[:, k0:k0 + Kk]),
                                              t(ent[:, k0:k0 + Kk]),
                                              torch.zeros(R * Kk + 1, dtype=torch.int64, device="cuda:0"), k0, K,
                                              ctx=comm_ctx, **kw)
    same(full, sh, ("ec", "oc", "ent"))
    # Map<K, Map<K2, MVReg>>: the nested generator's replicas with the far-future outer removes
    maps = O.nested_map_objects(30, K, 5, 6, seed=91, steps=400)
    V = max([len(ie.val.vals) for m in maps for e in m.entries.values() for ie in e.val.entries.values()] + [1])
    nd = O.nested_map_to_dense(maps, K, 5, 6, V)
    args = [t(nd[x]) for x in ("clock", "ec", "ic", "iec", "ivc", "ivv")]
    Dn2 = nd["def_row"].shape[0]
    kw2 = dict(def_off=[0, Dn2], def_row=torch.from_numpy(nd["def_row"].astype(np.int32)).cuda(),
               def_clock=t(nd["def_clock"]), def_keys=t(nd["def_keys"])) if Dn2 else {}
    ikw = dict(id_clock=t(nd["id_clock"]), id_keys=t(nd["id_keys"])) if nd["id_off"][-1] else {}
    full = cg.map.nested_lub_many(*args, t(nd["id_off"]), ctx=comm_ctx, **ikw, **kw2)
    R2 = nd["clock"].shape[0]
    # the inner removes' CSR restricted to this rank's keys: rows of (r, k) for k in the range
    off = nd["id_off"].astype(np.int64)
    rows, soff = [], [0]
    for r in range(R2):
        for k in range(k0, k0 + Kk):
            a, b = int(off[r * K + k]), int(off[r * K + k + 1])
            rows.extend(range(a, b))
            soff.append(len(rows))
    ikw2 = dict(id_clock=t(nd["id_clock"][rows]), id_keys=t(nd["id_keys"][rows])) if rows else {}
    sl = lambda x: t(nd[x][:, k0:k0 + Kk])  # noqa: E731
    sh = cg.shard.map_nested_lub_many_sharded(args[0], sl("ec"), sl("ic"), sl("iec"), sl("ivc"), sl("ivv"),
                                              t(np.array(soff, np.int64)), k0, K, ctx=comm_ctx, **ikw2, **kw2)
    np.testing.assert_array_equal(to_host(sh.clock), to_host(full.clock))
    hv = lambda x: x.cpu().numpy() if x.dtype == torch.int32 else to_host(x)  # noqa: E731
    for nm in ("ec", "ic", "iec", "ivc", "ivv", "nval", "id_n"):
        np.testing.assert_array_equal(hv(getattr(sh, nm)), hv(getattr(full, nm))[k0:k0 + Kk], err_msg=nm)
    idn = hv(full.id_n)[k0:k0 + Kk]  # (rows past a key's id_n are not written)
    for nm in ("id_clock", "id_keys"):
        a, b = hv(getattr(sh, nm)), hv(getattr(full, nm))[k0:k0 + Kk]
        for k in range(Kk):
            np.testing.assert_array_equal(a[k, :idn[k]], b[k, :idn[k]], err_msg=nm)
    assert idn.sum() > 0 or Kk == 0
    if Dn2:
        np.testing.assert_array_equal(sh.def_keep.cpu().numpy(), full.def_keep.cpu().numpy())
