"""World-size-2 gloo tests of the replica-sharded exchange (crdts_gpu.dist) on CPU.

The local fold is injected with the oracle (the checker) because this host has no GPU; what
is under test is the sharding and the exchange step: sign-biased MAX all-reduce for the
counter lattices, all-gather + re-merge for GSet."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_local(kind):
    import oracle as O

    def f(shard):
        a = shard.numpy().view(np.uint64)
        if a.ndim == 2:
            out = O.gset_fold(a)[0] if kind == "gset" else O.vclock_fold(a)[0]
        else:
            out = np.stack([O.gset_fold(x)[0] if kind == "gset" else O.vclock_fold(x)[0] for x in a])
        return torch.from_numpy(out.view(np.int64).copy())
    return f


def _worker(rank, world, port, kind, R, W, G, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "rust-crdt_amd"), os.path.join(here, "..", "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from crdts_gpu import dist as cdist
    full = O.synth_matrix(0x5EED0005, G * R, W, 1 if kind == "gset" else 0).reshape(G, R, W)
    lo, hi = cdist.shard_range(R, rank, world)
    shard = torch.from_numpy(full[:, lo:hi].view(np.int64).copy())
    if G == 1:
        shard = shard[0]
    out = cdist.lub_many_sharded(kind, shard, local_lub=_oracle_local(kind))
    if rank == 0:
        q.put(out.numpy().view(np.uint64).copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,R,W,G", [("gcounter", 101, 16, 1), ("vclock", 64, 9, 3),
                                         ("pncounter", 50, 24, 1), ("gset", 77, 5, 1), ("gset", 20, 3, 2)])
def test_sharded_lub_world2(kind, R, W, G):
    import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, R, W, G, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = O.synth_matrix(0x5EED0005, G * R, W, 1 if kind == "gset" else 0).reshape(G, R, W)
    fold = O.gset_fold if kind == "gset" else O.vclock_fold
    exp = np.stack([fold(full[g])[0] for g in range(G)])
    np.testing.assert_array_equal(got.reshape(G, W), exp)


def test_shard_range_partitions():
    from crdts_gpu.dist import shard_range
    for R in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(R, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == R
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


def test_sign_bias_preserves_unsigned_order():
    from crdts_gpu.dist import _bias
    vals = np.array([0, 1, 2**63 - 1, 2**63, 2**64 - 1, 12345], dtype=np.uint64)
    t = torch.from_numpy(vals.view(np.int64).copy())
    b = _bias(t)
    order_u = np.argsort(vals, kind="stable")
    order_s = np.argsort(b.numpy(), kind="stable")
    assert (order_u == order_s).all()


# ---- LWWReg and Orswot sharded exchanges -----------------------------------------------------
def _lww_local(m, v, init=None):
    import oracle as O
    mm, vv = m.numpy().view(np.uint64), v.numpy().view(np.uint64)
    G = mm.shape[0]
    om, ov, of = (np.zeros(G, dtype=np.uint64) for _ in range(3))
    for g in range(G):
        if init is None:
            acc, start = O.LWWReg(int(vv[g, 0]), int(mm[g, 0])), 1
        else:
            acc, start = O.LWWReg(int(init[1].numpy().view(np.uint64)[g]), int(init[0].numpy().view(np.uint64)[g])), 0
        first = 2**64 - 1
        for r in range(start, mm.shape[1]):
            try:
                acc.merge(O.LWWReg(int(vv[g, r]), int(mm[g, r])))
            except O.ConflictingMarker:
                first = min(first, r)
        om[g], ov[g], of[g] = acc.marker, acc.val, first
    t = lambda a: torch.from_numpy(a.view(np.int64).copy())
    return t(om), t(ov), t(of)


def _lww_worker(rank, world, port, G, R, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "rust-crdt_amd"), os.path.join(here, "..", "oracle"), here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from crdts_gpu import dist as cdist
    m = O.synth_matrix(41, G, R, 2) % np.uint64(6)
    v = O.synth_matrix(41, G, R, 3) % np.uint64(2)
    lo, hi = cdist.shard_range(R, rank, world)
    tm = torch.from_numpy(m[:, lo:hi].view(np.int64).copy())
    tv = torch.from_numpy(v[:, lo:hi].view(np.int64).copy())
    fm, fv, fc = cdist.lwwreg_lub_many_sharded(tm, tv, lo, local=_lww_local)
    if rank == 0:
        q.put((fm.numpy().copy(), fv.numpy().copy(), fc.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,G,R", [(2, 3, 40), (3, 2, 31)])
def test_lww_sharded_exact_conflicts(world, G, R):
    import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lww_worker, args=(r, world, port, G, R, q)) for r in range(world)]
    for p in procs:
        p.start()
    fm, fv, fc = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    m = O.synth_matrix(41, G, R, 2) % np.uint64(6)
    v = O.synth_matrix(41, G, R, 3) % np.uint64(2)
    for g in range(G):
        om, ov, of, _ = O.lwwreg_fold(m[g], v[g])
        got_fc = 2**64 - 1 if fc[g] == -1 else int(fc[g])
        assert (int(fm[g]), int(fv[g]), got_fc) == (om, ov, of)


def _orswot_local(clock, entries, def_off=None, def_clock=None, def_members=None):
    import oracle as O
    from crdts_gpu.orswot import OrswotLub
    c3 = clock.numpy().view(np.uint64)
    e4 = entries.numpy().view(np.uint64)
    G, _, A = c3.shape
    M = e4.shape[2]
    Mw = (M + 63) // 64
    oc = np.zeros((G, A), np.uint64)
    oe = np.zeros((G, M, A), np.uint64)
    D = 0 if def_off is None else int(def_off[-1])
    keep = np.zeros(D, np.uint8)
    mem = np.zeros((D, Mw), np.uint64)
    dcl = def_clock.numpy().view(np.uint64) if D else None
    dmm = def_members.numpy().view(np.uint64) if D else None
    for g in range(G):
        lo, hi = (int(def_off[g]), int(def_off[g + 1])) if D else (0, 0)
        c, e, surv = O.dense_orswot_lub(c3[g], e4[g], dcl[lo:hi] if D else np.zeros((0, A), np.uint64),
                                        dmm[lo:hi] if D else np.zeros((0, Mw), np.uint64))
        oc[g], oe[g] = c, e
        for d in range(lo, hi):  # representative = first survivor with that clock
            key = tuple(int(x) for x in dcl[d])
            for k, ms in surv:
                if k == key and not any(tuple(int(x) for x in dcl[d2]) == key and keep[d2] for d2 in range(lo, d)):
                    keep[d] = 1
                    for mm in ms:
                        mem[d, mm // 64] |= np.uint64(1) << np.uint64(mm % 64)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy())
    return OrswotLub(t(oc), t(oe), torch.from_numpy(keep), t(mem))


def _orswot_worker(rank, world, port, R, M, A, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "rust-crdt_amd"), os.path.join(here, "..", "oracle"), here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from crdts_gpu import dist as cdist
    clock, entries, off, dcl, dmem = O.gen_orswot(99, R, M, A, kmax=10)
    lo, hi = cdist.shard_range(R, rank, world)
    d0, d1 = int(off[lo]), int(off[hi])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy())
    res = cdist.orswot_lub_many_sharded(t(clock[lo:hi][None]), t(entries[lo:hi][None]), t(dcl[d0:d1]),
                                        t(dmem[d0:d1]), torch.zeros(d1 - d0, dtype=torch.int64),
                                        local=_orswot_local)
    if rank == 0:
        from crdts_gpu.orswot import deferred_set
        D = res.def_keep.shape[0] if res.def_keep is not None else 0
        allcl = torch.cat([t(dcl)]) if D else None
        # the re-merge pools deferred removes in rank order == original order here
        dset = deferred_set(allcl, res.def_keep, res.def_members) if D else set()
        q.put((res.clock.numpy().copy(), res.entries.numpy().copy(), dset))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_orswot_sharded_world(world):
    import oracle as O
    R, M, A = 13, 20, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_orswot_worker, args=(r, world, port, R, M, A, q)) for r in range(world)]
    for p in procs:
        p.start()
    c, e, dset = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    clock, entries, off, dcl, dmem = O.gen_orswot(99, R, M, A, kmax=10)
    oc, oe, odef, _ = O.orswot_fold(clock, entries, off, dcl, dmem)
    np.testing.assert_array_equal(c.view(np.uint64)[0], oc)
    np.testing.assert_array_equal(e.view(np.uint64)[0], oe)
    assert dset == odef


def _map_local(clock, ec, vclk, vval, vout=4, def_off=None, def_row=None, def_clock=None, def_keys=None):
    """Oracle stand-in for crdts_gpu.map.lub_many (one group), same deferred-output convention:
    keep[d] = d is the first surviving remove with its rm clock (survival: !(rm <= final clock),
    map.rs:336-345), def_keys[d] = the union of the key sets of the survivors with that clock."""
    import oracle as O
    from crdts_gpu.map import MapLub
    c = clock.numpy().view(np.uint64)[0]
    e, vc, vv = (x.numpy().view(np.uint64)[0] for x in (ec, vclk, vval))
    K = e.shape[1]
    Kw = (K + 63) // 64
    D = 0 if def_off is None else int(def_off[-1])
    rows = def_row.numpy().astype(np.int64) if D else None
    dcl = def_clock.numpy().view(np.uint64) if D else None
    dk = def_keys.numpy().view(np.uint64) if D else None
    oc, oe, ovc, ovv, on, _, _ = O.map_fold(c, e, vc, vv, rows, dcl, dk, vout)
    keep = np.zeros(D, np.uint8)
    keys = np.zeros((D, Kw), np.uint64)
    for d in range(D):
        if np.all(dcl[d] <= oc):
            continue
        first = next(d2 for d2 in range(D) if np.array_equal(dcl[d2], dcl[d]))
        keep[first] = 1
        keys[first] |= dk[d]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy())  # noqa: E731
    return MapLub(t(oc[None]), t(oe[None]), t(ovc[None]), t(ovv[None]), torch.from_numpy(on[None].astype(np.int32)),
                  torch.zeros(1, dtype=torch.int32), torch.from_numpy(keep) if D else None, t(keys) if D else None)


def _map_data(seed):
    import oracle as O
    maps = O.gen_map_replicas(seed, 30, 21, 5, steps=260, p_rm=0.3, p_up=0.4)
    return O.map_to_dense(maps, 21, 5, O.max_vals(maps))


def _map_worker(rank, world, port, seed, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "rust-crdt_amd"), os.path.join(here, "..", "oracle"), here):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from crdts_gpu import dist as cdist
    d = _map_data(seed)
    K = d["ec"].shape[1]
    k0, k1 = cdist.shard_range(K, rank, world)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy())  # noqa: E731
    D = d["def_row"].shape[0]
    kw = dict(def_off=[0, D], def_row=torch.from_numpy(d["def_row"].astype(np.int32)),
              def_clock=t(d["def_clock"]), def_keys=t(d["def_keys"])) if D else {}
    res = cdist.map_lub_many_sharded(t(d["clock"][None]), t(d["ec"][None, :, k0:k1]),
                                     t(d["vclk"][None, :, k0:k1]), t(d["vval"][None, :, k0:k1]), k0, K,
                                     vout=8, local=_map_local, **kw)
    q.put((rank, k0, res.clock.numpy().copy(), res.ec.numpy().copy(), res.vclk.numpy().copy(),
           res.vval.numpy().copy(), res.nval.numpy().copy(),
           None if res.def_keep is None else res.def_keep.numpy().copy(),
           None if res.def_keys is None else res.def_keys.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,seed", [(2, 3), (3, 4)])
def test_map_key_sharded_world(world, seed):
    """Key-sharded Map fold: the ranks' key ranges assemble to the oracle's whole left fold, and
    the exchanged surviving removes equal the oracle's deferred set."""
    import oracle as O
    from crdts_gpu.orswot import deferred_set
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_map_worker, args=(r, world, port, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    d = _map_data(seed)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"], 8)
    assert d["def_row"].shape[0] > 0
    for rank, k0, c, e, vc, vv, nv, keep, keys in outs:
        n = e.shape[1]
        np.testing.assert_array_equal(c.view(np.uint64)[0], exp[0])
        np.testing.assert_array_equal(e.view(np.uint64)[0], exp[1][k0:k0 + n])
        np.testing.assert_array_equal(vc.view(np.uint64)[0], exp[2][k0:k0 + n])
        np.testing.assert_array_equal(vv.view(np.uint64)[0], exp[3][k0:k0 + n])
        np.testing.assert_array_equal(nv[0], exp[4][k0:k0 + n])
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy())  # noqa: E731
        got = deferred_set(t(d["def_clock"]), torch.from_numpy(keep), torch.from_numpy(keys))
        assert got == exp[5]
