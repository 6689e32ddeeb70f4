"""GPU parity: serde wire format (bincode 1.x) ingest / egress (crdt_*_ingest, crdt_*_egress;
SURVEY §8f row 1) against the oracle's bincode restatement (oracle.bc_* / unbc_*):
  * ingest of random frames equals the dense layout built on the host, byte-exact egress of
    canonical frames, order-free Orswot maps;
  * end to end: serialized replicas -> ingest -> lub_many -> egress -> decode == the oracle's
    fold of the same replicas (VClock, PNCounter, GSet, LWWReg, Orswot with deferred removes);
  * the reference's KATs with every merge routed through bytes (serialize both states, ingest,
    merge on the GPU, egress, decode);
  * malformed frames (truncated, trailing bytes, misaligned) and ids missing from a dictionary
    are reported per state, never read past the frame."""
import numpy as np
import pytest
import torch

import kat_runner as K
import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import wire  # noqa: E402


def dev_bytes(blob: bytes):
    return torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda() if blob else torch.zeros(4, dtype=torch.uint8,
                                                                                                  device="cuda")


def dev_off(off):
    return torch.tensor(off, dtype=torch.int64, device="cuda")


def host_frames(data: torch.Tensor, off: torch.Tensor):
    b = bytes(data.cpu().numpy().tobytes())
    o = off.cpu().numpy().tolist()
    return [b[o[i]:o[i + 1]] for i in range(len(o) - 1)]


def actor_dict(rng, A):
    ids = np.sort(rng.choice(2**32 - 1, size=A, replace=False)).astype(np.uint32)
    return ids, torch.from_numpy(ids.view(np.int32).copy()).cuda()


def u64_dict(rng, M):
    ids = np.sort(rng.choice(2**62, size=M, replace=False)).astype(np.uint64)
    return ids, torch.from_numpy(ids.view(np.int64).copy()).cuda()


def rand_rows(rng, N, A, p=0.6):
    rows = rng.integers(1, 2**63, size=(N, A), dtype=np.uint64)
    rows[rng.random((N, A)) > p] = 0
    rows[rng.integers(0, N, size=max(1, N // 10))] = 0  # some empty clocks
    return rows


def row_dots(row, ids):
    return {int(ids[a]): int(v) for a, v in enumerate(row) if v}


@pytest.mark.parametrize("N,A", [(300, 70), (64, 1), (17, 1024), (1, 4096)])
def test_vclock_ingest_egress(gpu_ctx, N, A):
    rng = np.random.default_rng(N + A)
    ids, dd = actor_dict(rng, A)
    rows = rand_rows(rng, N, A)
    blob, off = O.frames([O.bc_vclock(row_dots(r, ids)) for r in rows])
    got, st = wire.vclock_ingest(dev_bytes(blob), dev_off(off), dd, ctx=gpu_ctx)
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(to_host(got), rows)
    eoff, edata = wire.vclock_egress(got, dd, ctx=gpu_ctx)
    assert eoff.cpu().tolist() == off
    assert bytes(edata.cpu().numpy().tobytes()) == blob  # canonical frames round-trip byte for byte


def test_pncounter_gset_lwwreg_round_trip(gpu_ctx):
    rng = np.random.default_rng(5)
    N, A, U = 200, 33, 300
    ids, dd = actor_dict(rng, A)
    p, n = rand_rows(rng, N, A), rand_rows(rng, N, A, 0.3)
    blob, off = O.frames([O.bc_pncounter(row_dots(p[i], ids), row_dots(n[i], ids)) for i in range(N)])
    got, st = wire.pncounter_ingest(dev_bytes(blob), dev_off(off), dd, ctx=gpu_ctx)
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(to_host(got), np.concatenate([p, n], axis=1))
    eoff, edata = wire.pncounter_egress(got, dd, ctx=gpu_ctx)
    assert bytes(edata.cpu().numpy().tobytes()) == blob
    # GSet<u64>
    eids, ed = u64_dict(rng, U)
    sets = [set(int(x) for x in rng.choice(eids, size=int(rng.integers(0, 40)), replace=False)) for _ in range(N)]
    blob, off = O.frames([O.bc_gset(s) for s in sets])
    bm, st = wire.gset_ingest(dev_bytes(blob), dev_off(off), ed, ctx=gpu_ctx)
    assert (st.cpu().numpy() == 0).all()
    pos = {int(x): i for i, x in enumerate(eids)}
    exp = np.zeros((N, (U + 63) // 64), np.uint64)
    for i, s in enumerate(sets):
        for x in s:
            exp[i, pos[x] // 64] |= np.uint64(1) << np.uint64(pos[x] % 64)
    np.testing.assert_array_equal(to_host(bm), exp)
    eoff, edata = wire.gset_egress(bm, ed, ctx=gpu_ctx)
    assert bytes(edata.cpu().numpy().tobytes()) == blob
    # LWWReg<u64, u64>
    vals, marks = rng.integers(0, 2**63, N).astype(np.uint64), rng.integers(0, 2**63, N).astype(np.uint64)
    blob, off = O.frames([O.bc_lwwreg(v, m) for v, m in zip(vals, marks)])
    m, v, st = wire.lwwreg_ingest(dev_bytes(blob), dev_off(off), ctx=gpu_ctx)
    assert (st.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(to_host(m), marks)
    np.testing.assert_array_equal(to_host(v), vals)
    eoff, edata = wire.lwwreg_egress(m, v, ctx=gpu_ctx)
    assert bytes(edata.cpu().numpy().tobytes()) == blob


@pytest.fixture(params=["wwalk=1,wfill=1", "wwalk=1,wfill=0", "wwalk=0"], ids=["walk_fill", "walk", "chain"])
def octx(request, gpu_ctx):
    """Every Orswot ingest pass-1 kernel: the walk with filler waves zeroing the rows beside it (round 4
    default), the walk after a separate zero-fill pass, and the per-state chain."""
    gpu_ctx.tune(request.param)
    yield gpu_ctx
    gpu_ctx.tune("wwalk=1,wfill=1")


def orswot_objects(seed, R, M, A):
    """gen_orswot replicas as (clock, entries, deferred) dicts over dense indices."""
    clock, entries, off, dcl, dmem = O.gen_orswot(seed, R, M, A, kmax=12, p_def=0.5)
    out = []
    for r in range(R):
        ent = {m: {a: int(v) for a, v in enumerate(entries[r, m]) if v} for m in range(M) if entries[r, m].any()}
        de = {}
        for d in range(int(off[r]), int(off[r + 1])):
            key = tuple((a, int(v)) for a, v in enumerate(dcl[d]) if v)
            de.setdefault(key, set()).update(O.bitmap_members(dmem[d]))
        out.append(({a: int(v) for a, v in enumerate(clock[r]) if v}, ent, de))
    return out, (clock, entries, off, dcl, dmem)


def orswot_blob(states, aids, mids, rng):
    blobs = []
    for c, ent, de in states:
        ent_ids = {int(mids[m]): {int(aids[a]): v for a, v in e.items()} for m, e in ent.items()}
        order = list(ent_ids)
        rng.shuffle(order)  # HashMap: any order
        dlist = [({int(aids[a]): v for a, v in k}, [int(mids[m]) for m in ms]) for k, ms in de.items()]
        blobs.append(O.bc_orswot({int(aids[a]): v for a, v in c.items()}, ent_ids, dlist, order=order))
    return O.frames(blobs)


@pytest.mark.parametrize("R,M,A", [(40, 90, 9), (12, 70, 64), (10, 40, 65), (8, 30, 1)])
def test_orswot_ingest_egress(octx, R, M, A):
    """A <= 64 takes the batched lane-per-actor egress, A > 64 the generic row loop."""
    rng = np.random.default_rng(11 + A)
    states, (clock, entries, off, dcl, dmem) = orswot_objects(3, R, M, A)
    aids, ad = actor_dict(rng, A)
    mids, md = u64_dict(rng, M)
    blob, foff = orswot_blob(states, aids, mids, rng)
    res = wire.orswot_ingest(dev_bytes(blob), dev_off(foff), ad, md, ctx=octx)
    assert (res.status.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(to_host(res.clock), clock)
    np.testing.assert_array_equal(to_host(res.entries), entries)
    # pooled removes in state order; within a state, frame order (= the object's dict order)
    got_def = [set() for _ in range(R)]
    doff = res.def_off.cpu().numpy()
    gd, gm = to_host(res.def_clock), to_host(res.def_members)
    for r in range(R):
        for d in range(int(doff[r]), int(doff[r + 1])):
            got_def[r].add((tuple((a, int(v)) for a, v in enumerate(gd[d]) if v), O.bitmap_members(gm[d])))
    assert got_def == [{(k, frozenset(ms)) for k, ms in de.items()} for _, _, de in states]
    assert int(doff[-1]) > 0
    # egress of the ingested states decodes to the same objects
    eoff, edata = wire.orswot_egress(res.clock, res.entries, ad, md, res.def_off, res.def_clock, res.def_members,
                                     ctx=octx)
    for r, fr in enumerate(host_frames(edata, eoff)):
        c, e, d, pos = O.unbc_orswot(fr)
        assert pos == len(fr)
        c0, e0, d0 = states[r]
        assert c == {int(aids[a]): v for a, v in c0.items()}
        assert e == {int(mids[m]): {int(aids[a]): v for a, v in x.items()} for m, x in e0.items()}
        assert d == {tuple(sorted((int(aids[a]), v) for a, v in k)): {int(mids[m]) for m in ms} for k, ms in d0.items()}


def test_end_to_end_orswot_fold_through_bytes(octx):
    """R serialized replicas -> ingest -> lub_many -> egress -> decode == the oracle fold."""
    rng = np.random.default_rng(12)
    R, M, A = 64, 120, 16
    states, raw = orswot_objects(8, R, M, A)
    aids, ad = actor_dict(rng, A)
    mids, md = u64_dict(rng, M)
    blob, foff = orswot_blob(states, aids, mids, rng)
    res = wire.orswot_ingest(dev_bytes(blob), dev_off(foff), ad, md, ctx=octx)
    D = res.def_clock.shape[0]
    lub = cg.orswot.lub_many(res.clock, res.entries, def_off=[0, D], def_clock=res.def_clock,
                             def_members=res.def_members, ctx=octx)
    one = torch.tensor([0, D], dtype=torch.int64, device="cuda")
    eoff, edata = wire.orswot_egress(lub.clock[None].contiguous(), lub.entries[None].contiguous(), ad, md, one,
                                     res.def_clock, lub.def_members, lub.def_keep, ctx=octx)
    c, e, d, pos = O.unbc_orswot(host_frames(edata, eoff)[0])
    oc, oe, odef, _ = O.orswot_fold(*raw)
    assert c == {int(aids[a]): int(v) for a, v in enumerate(oc) if v}
    assert e == {int(mids[m]): {int(aids[a]): int(v) for a, v in enumerate(oe[m]) if v} for m in range(M) if oe[m].any()}
    assert d == {tuple(sorted((int(aids[a]), v) for a, v in enumerate(k) if v)): {int(mids[m]) for m in ms}
                 for k, ms in odef}
    assert odef


def test_end_to_end_counters_through_bytes(gpu_ctx):
    rng = np.random.default_rng(13)
    R, A = 500, 64
    ids, dd = actor_dict(rng, A)
    rows = rand_rows(rng, R, 2 * A)
    blob, off = O.frames([O.bc_pncounter(row_dots(r[:A], ids), row_dots(r[A:], ids)) for r in rows])
    dense, st = wire.pncounter_ingest(dev_bytes(blob), dev_off(off), dd, ctx=gpu_ctx)
    lub = cg.pncounter.lub_many(dense, ctx=gpu_ctx)
    eoff, edata = wire.pncounter_egress(lub[None], dd, ctx=gpu_ctx)
    fr = host_frames(edata, eoff)[0]
    p, pos = O.unbc_vclock(fr)
    n, pos = O.unbc_vclock(fr, pos)
    exp, _ = O.pncounter_fold(rows)
    assert p == row_dots(exp[:A], ids) and n == row_dots(exp[A:], ids) and pos == len(fr)


def test_malformed_frames_and_missing_ids(gpu_ctx):
    rng = np.random.default_rng(14)
    A = 8
    ids, dd = actor_dict(rng, A)
    good = O.bc_vclock({int(ids[1]): 5, int(ids[3]): 7})
    missing = O.bc_vclock({int(ids[1]): 5, int(ids[2]) + 1: 9})   # an actor outside the dictionary
    truncated = good[:-4]
    trailing = good + b"\x00\x00\x00\x00"
    lying = b"\xff" + good[1:]                                      # a length far past the frame
    parts = [good, missing, truncated, trailing, lying]
    blob = b"".join(parts)
    off = np.cumsum([0] + [len(x) for x in parts]).tolist()
    rows, st = wire.vclock_ingest(dev_bytes(blob), dev_off(off), dd, ctx=gpu_ctx)
    assert st.cpu().tolist() == [0, 2, 1, 1, 1]
    r = to_host(rows)
    assert r[0, 1] == 5 and r[0, 3] == 7 and r[1, 1] == 5 and r[1].sum() == 5
    # a misaligned frame offset is malformed (frames are whole 4-byte words)
    rows, st = wire.vclock_ingest(dev_bytes(good + good), dev_off([0, 2, len(good) * 2]), dd, ctx=gpu_ctx)
    assert st.cpu().tolist() == [1, 1]


def test_orswot_lying_deferred_count_only_breaks_its_frame(octx):
    """a frame whose deferred-remove count is far larger than its bytes could hold must be
    malformed on its own (status bit 0, no removes), not shift / wrap the pooled def_off of every
    later state or make the wrapper allocate a (count, A) buffer."""
    rng = np.random.default_rng(15)
    R, M, A = 6, 50, 8
    states, _ = orswot_objects(5, R, M, A)
    with_def = [s for s in states if s[2]]
    assert len(with_def) >= 2
    states = with_def[:2] + [s for s in states if not s[2]] + with_def[2:]
    aids, ad = actor_dict(rng, A)
    mids, md = u64_dict(rng, M)
    blob, foff = orswot_blob(states, aids, mids, rng)
    fo = [int(x) for x in foff]
    frames = [blob[fo[i]:fo[i + 1]] for i in range(len(fo) - 1)]
    c0, e0, _ = states[2]
    empty_def = O.bc_orswot({int(aids[a]): v for a, v in c0.items()},
                            {int(mids[m]): {int(aids[a]): v for a, v in e.items()} for m, e in e0.items()}, [])
    assert empty_def[-8:] == bytes(8)  # the trailing u64 is the deferred count (0)
    lying = empty_def[:-8] + (1 << 40).to_bytes(8, "little")
    parts = [bytes(frames[0]), lying, bytes(frames[1])]
    blob2 = b"".join(parts)
    off = np.cumsum([0] + [len(x) for x in parts]).tolist()
    res = wire.orswot_ingest(dev_bytes(blob2), dev_off(off), ad, md, ctx=octx)
    assert res.status.cpu().tolist()[1] & 1 and res.status.cpu().tolist()[0] == 0 and res.status.cpu().tolist()[2] == 0
    doff = res.def_off.cpu().numpy()
    n0, n1 = len(states[0][2]), len(states[1][2])
    assert doff.tolist() == [0, n0, n0, n0 + n1]
    gd, gm = to_host(res.def_clock), to_host(res.def_members)
    for r, st_ in ((0, 0), (2, 1)):
        got = {(tuple((a, int(v)) for a, v in enumerate(gd[d]) if v), O.bitmap_members(gm[d]))
               for d in range(int(doff[r]), int(doff[r + 1]))}
        assert got == {(k, frozenset(ms)) for k, ms in states[st_][2].items()}


# ---- the reference's KATs with every merge through bytes -------------------------------------
def _ids(values):
    """Deterministic u32 / u64 ids for the KATs' actors and members (strings or ints)."""
    vs = sorted(set(values), key=lambda x: (str(type(x)), x))
    return {v: i + 1 for i, v in enumerate(vs)}


def wire_merge(dst, src, kind):
    if kind in ("vclock", "gcounter", "pncounter"):
        def parts(x):
            if kind == "vclock":
                return [x.dots]
            if kind == "gcounter":
                return [x.inner.dots]
            return [x.p.inner.dots, x.n.inner.dots]
        pa, pb = parts(dst), parts(src)
        amap = _ids([a for d in pa + pb for a in d])
        inv = {v: k for k, v in amap.items()}
        aids = np.array(sorted(amap.values()) or [1], np.uint32)
        dd = torch.from_numpy(aids.view(np.int32).copy()).cuda()
        enc = (lambda ds: b"".join(O.bc_vclock({amap[a]: c for a, c in d.items()}) for d in ds))
        blob, off = O.frames([enc(pa), enc(pb)])
        ing = wire.pncounter_ingest if kind == "pncounter" else wire.vclock_ingest
        egr = wire.pncounter_egress if kind == "pncounter" else wire.vclock_egress
        rows, st = ing(dev_bytes(blob), dev_off(off), dd)
        assert (st.cpu().numpy() == 0).all()
        mod = {"vclock": cg.vclock, "gcounter": cg.gcounter, "pncounter": cg.pncounter}[kind]
        eoff, edata = egr(mod.lub_many(rows)[None], dd)
        fr = host_frames(edata, eoff)[0]
        out, pos = O.unbc_vclock(fr)
        dec = [out]
        if kind == "pncounter":
            dec.append(O.unbc_vclock(fr, pos)[0])
        back = [{inv[a]: c for a, c in d.items()} for d in dec]
        if kind == "vclock":
            dst.dots = back[0]
        elif kind == "gcounter":
            dst.inner.dots = back[0]
        else:
            dst.p.inner.dots, dst.n.inner.dots = back
        return dst
    if kind == "orswot":
        amap = _ids([a for s in (dst, src) for c in [s.clock] + list(s.entries.values()) + list(s.deferred)
                     for a in c.dots])
        mmap = _ids([m for s in (dst, src) for m in list(s.entries) + [x for ms in s.deferred.values() for x in ms]])
        ainv, minv = {v: k for k, v in amap.items()}, {v: k for k, v in mmap.items()}
        aids = np.array(sorted(amap.values()) or [1], np.uint32)
        mids = np.array(sorted(mmap.values()) or [1], np.uint64)
        ad = torch.from_numpy(aids.view(np.int32).copy()).cuda()
        md = torch.from_numpy(mids.view(np.int64).copy()).cuda()
        blobs = [O.bc_orswot({amap[a]: c for a, c in s.clock.dots.items()},
                             {mmap[m]: {amap[a]: c for a, c in e.dots.items()} for m, e in s.entries.items()},
                             [({amap[a]: c for a, c in k.dots.items()}, [mmap[m] for m in ms])
                              for k, ms in s.deferred.items()]) for s in (dst, src)]
        blob, off = O.frames(blobs)
        res = wire.orswot_ingest(dev_bytes(blob), dev_off(off), ad, md)
        assert (res.status.cpu().numpy() == 0).all()
        D = res.def_clock.shape[0]
        kw = dict(def_off=[0, D], def_clock=res.def_clock, def_members=res.def_members) if D else {}
        lub = cg.orswot.lub_many(res.clock, res.entries, **kw)
        one = torch.tensor([0, D], dtype=torch.int64, device="cuda")
        eoff, edata = wire.orswot_egress(lub.clock[None].contiguous(), lub.entries[None].contiguous(), ad, md,
                                         one if D else None, res.def_clock, lub.def_members, lub.def_keep)
        c, e, d, _ = O.unbc_orswot(host_frames(edata, eoff)[0])
        out = O.Orswot()
        out.clock = O.VClock({ainv[a]: v for a, v in c.items()})
        out.entries = {minv[m]: O.VClock({ainv[a]: v for a, v in x.items()}) for m, x in e.items()}
        out.deferred = {O.VClock({ainv[a]: v for a, v in k}): {minv[m] for m in ms} for k, ms in d.items()}
        return out
    from test_gpu_kat import gpu_merge
    return gpu_merge(dst, src, kind)


CASES = [c for f in ("kat_vclock.json", "kat_counters.json", "kat_orswot.json")
         for c in K.load_cases(f) if any(s[0] in ("merge", "merge_err") for s in c["steps"])]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_kat_merges_through_the_wire(gpu_ctx, case):
    K.run_case(case, merge_hook=wire_merge)


# ---- Map<u32, MVReg<u64>> (BASELINE config 4's type) ---------------------------------------------
@pytest.fixture(params=[1, 0], ids=["walk", "chain"])
def mctx(request, gpu_ctx):
    """Both Map ingest kernels: the walk + batched parse (default) and the per-state dependent chain."""
    gpu_ctx.tune(f"wwalk={request.param}")
    yield gpu_ctx
    gpu_ctx.tune("wwalk=1")


def map_wire_form(m, aids, kids):
    """oracle Map over dense actor / key indices -> bc_map arguments over the u32 ids."""
    tr = lambda vc: {int(aids[a]): int(v) for a, v in vc.dots.items() if v}  # noqa: E731
    entries = {int(kids[k]): (tr(e.clock), [(tr(c), int(v)) for c, v in e.val.vals]) for k, e in m.entries.items()}
    deferred = [(tr(rm), [int(kids[k]) for k in keys]) for rm, keys in m.deferred.items()]
    return tr(m.clock), entries, deferred


def map_decoded(m, aids, kids):
    c, e, d = map_wire_form(m, aids, kids)
    return c, e, {tuple(sorted(rm.items())): set(ks) for rm, ks in d}


def map_blob(maps, aids, kids):
    return O.frames([O.bc_map(*map_wire_form(m, aids, kids)) for m in maps])


@pytest.mark.parametrize("A,V", [(5, 3), (64, 2), (70, 2), (5, 5)])
def test_map_ingest_egress(mctx, A, V):
    """A <= 64 with V <= 4 takes the batched egress, the others the generic loop."""
    from test_gpu_merge_batch import arbitrary_maps, map_side
    rng = np.random.default_rng(41 + A + V)
    N, K = 40, 9
    maps = arbitrary_maps(rng, N, K, A, V, 4)
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)  # u32 keys
    blob, off = map_blob(maps, aids, kids)
    Dcap = max(1, max(len(m.deferred) for m in maps))
    st, status = wire.map_ingest(dev_bytes(blob), dev_off(off), ad, kd, V, Dcap, ctx=mctx)
    assert (status.cpu().numpy() == 0).all()
    exp = map_side(maps, K, A, V, Dcap)
    for nm in exp._fields:
        np.testing.assert_array_equal(getattr(st, nm).cpu().numpy(), getattr(exp, nm).cpu().numpy(), err_msg=nm)
    assert int(st.def_count.sum()) > 0 and int((st.vclk != 0).any(dim=3).sum()) > 0
    eoff, edata = wire.map_egress(st, ad, kd, ctx=mctx)
    assert eoff.cpu().tolist() == off
    assert bytes(edata.cpu().numpy().tobytes()) == blob  # canonical frames round-trip byte for byte


def test_map_merge_batch_through_bytes(mctx):
    """Serialized pairs -> ingest -> merge_batch -> egress -> decode == the oracle's Map::merge."""
    from test_gpu_merge_batch import replay_maps
    rng = np.random.default_rng(42)
    N, K, n_origins = 24, 12, 5
    maps = replay_maps(7, 2 * N, n_origins, K, 200)
    lhs, rhs = maps[:N], maps[N:]
    exp = []
    for a, b in zip(lhs, rhs):
        x = a.copy()
        x.merge(b.copy())
        exp.append(x)
    aids, ad = actor_dict(rng, n_origins)
    kids, kd = actor_dict(rng, K)
    V = max(1, O.max_vals(exp), O.max_vals(lhs), O.max_vals(rhs))
    Dcap = max(1, max(len(m.deferred) for m in list(lhs) + list(rhs) + exp))
    b1, o1 = map_blob(lhs, aids, kids)
    b2, o2 = map_blob(rhs, aids, kids)
    s1, st1 = wire.map_ingest(dev_bytes(b1), dev_off(o1), ad, kd, V, Dcap, ctx=mctx)
    s2, st2 = wire.map_ingest(dev_bytes(b2), dev_off(o2), ad, kd, V, Dcap, ctx=mctx)
    assert (st1.cpu().numpy() == 0).all() and (st2.cpu().numpy() == 0).all()
    status = cg.map.merge_batch(s1, s2, ctx=mctx).cpu().numpy()
    assert (status == 0).all(), status
    eoff, edata = wire.map_egress(s1, ad, kd, ctx=mctx)
    for i, fr in enumerate(host_frames(edata, eoff)):
        c, e, d, pos = O.unbc_map(fr)
        assert pos == len(fr)
        assert (c, e, d) == map_decoded(exp[i], aids, kids), i
    assert sum(len(x.entries) for x in exp) > 0 and sum(len(x.deferred) for x in exp) > 0


def test_map_malformed_missing_and_capacity(mctx):
    rng = np.random.default_rng(43)
    K, A = 4, 3
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)
    a = lambda i: int(aids[i])  # noqa: E731
    good = O.bc_map({a(0): 3}, {int(kids[1]): ({a(0): 3}, [({a(0): 3}, 7)])}, [({a(1): 5}, [int(kids[2])])])
    missing_key = O.bc_map({a(0): 1}, {int(kids[-1]) + 1 if int(kids[-1]) < 2**32 - 1 else 0: ({a(0): 1}, [])}, [])
    three_vals = O.bc_map({a(0): 2, a(1): 2, a(2): 2},
                          {int(kids[0]): ({a(0): 2, a(1): 2, a(2): 2}, [({a(0): 2}, 1), ({a(1): 2}, 2), ({a(2): 2}, 3)])},
                          [])
    blobs = [good, good[:-4], good + b"\0\0\0\0", missing_key, three_vals]
    blob, off = O.frames(blobs)
    st, status = wire.map_ingest(dev_bytes(blob), dev_off(off), ad, kd, 2, 1, ctx=mctx)
    s = status.cpu().numpy().tolist()
    assert s[0] == 0
    assert s[1] & wire.BAD and s[2] & wire.BAD
    assert s[3] == wire.MISSING
    assert s[4] == wire.CAP  # a third value with V = 2 slots: dropped and reported
    assert to_host(st.vval)[4, 0].tolist() == [1, 2]


@pytest.mark.parametrize("walk", [1, 0])
def test_map_ingest_large_frames(walk):
    """Config-4-shaped frames (1,024 keys x 32 actors, ~80 KiB each): synthetic states -> egress ->
    ingest is the identity; truncated / extended copies of large frames are reported as malformed
    and leave the other states' rows exact.  Both ingest kernels (walk: the frame streams through
    the LDS ring in 1-KiB windows; chain)."""
    from crdts_gpu import synth
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    ctx.tune(f"wwalk={walk}")
    dev = "cuda"
    R, K, A, V = 24, 1024, 32, 2
    inp = synth.map_replicas(ctx, R, K, A, V, 0x5EED0004, kmax=256, p_def=0.3)
    rows = inp.def_row.cpu().numpy().astype(np.int64)
    cnt = np.bincount(rows, minlength=R).astype(np.int32)
    Dcap = max(1, int(cnt.max()))
    Kw = (K + 63) // 64
    dcl = torch.zeros((R, Dcap, A), dtype=torch.int64, device=dev)
    dks = torch.zeros((R, Dcap, Kw), dtype=torch.int64, device=dev)
    slot = np.arange(rows.shape[0]) - np.searchsorted(rows, rows)
    rt, st_ = torch.from_numpy(rows).to(dev), torch.from_numpy(slot).to(dev)
    dcl[rt, st_] = inp.def_clock
    dks[rt, st_] = inp.def_keys
    states = cg.map.MapStates(inp.clock, inp.ec, inp.vclk, inp.vval, dcl, dks, torch.from_numpy(cnt).to(dev))
    actors = torch.arange(1, A + 1, dtype=torch.int32, device=dev) * 5
    keys = torch.arange(1, K + 1, dtype=torch.int32, device=dev) * 11
    off, frames = wire.map_egress(states, actors, keys, ctx=ctx)
    o = off.cpu().numpy()
    assert int(np.diff(o).min()) > 16 * 1024  # every frame spans several 8-KiB windows
    back, status = wire.map_ingest(frames, off, actors, keys, V, Dcap, ctx=ctx)
    assert (status.cpu().numpy() == 0).all()
    for f in states._fields:
        assert torch.equal(getattr(back, f), getattr(states, f)), f
    # malformed copies: frame 0 truncated in its last window, frame 1 with 8 trailing bytes
    fr = host_frames(frames, off)
    cut = fr[0][:len(fr[0]) - 12]
    blob, noff = O.frames([cut, fr[1] + b"\0" * 8, fr[2]])
    st2, s2 = wire.map_ingest(dev_bytes(blob), dev_off(noff), actors, keys, V, Dcap, ctx=ctx)
    s = s2.cpu().numpy().tolist()
    assert s[0] & wire.BAD and s[1] & wire.BAD and s[2] == 0
    for f in states._fields:
        assert torch.equal(getattr(st2, f)[2], getattr(states, f)[2]), f


def test_orswot_malformed_frames(octx):
    """Malformed Orswot frames set their own status bits and leave every other frame's rows exact:
    a member or an actor missing from its dictionary (bit 1, the rest parsed), a truncated frame,
    an entry count and a record count far past the frame (bit 0)."""
    rng = np.random.default_rng(22)
    R, M, A = 4, 40, 8
    states, (clock, entries, off, dcl, dmem) = orswot_objects(7, R, M, A)
    aids, ad = actor_dict(rng, A)
    mids, md = u64_dict(rng, M)
    blob, foff = orswot_blob(states, aids, mids, rng)
    fo = [int(x) for x in foff]
    good = [bytes(blob[fo[i]:fo[i + 1]]) for i in range(R)]
    c0, e0, _ = states[0]
    cl = {int(aids[a]): v for a, v in c0.items()}
    ent = {int(mids[m]): {int(aids[a]): v for a, v in e.items()} for m, e in e0.items()}
    m_any = next(iter(ent))
    bad_member = dict(ent)
    bad_member[int(mids.max()) + 1] = {int(aids[0]): 1}            # not in the member dictionary
    bad_actor = dict(ent)
    bad_actor[m_any] = {**ent[m_any], int(aids.max()) + 1: 3}      # an actor outside the dictionary
    fr_member = O.bc_orswot(cl, bad_member, [])
    fr_actor = O.bc_orswot(cl, bad_actor, [])
    truncated = good[1][:-4]
    # the entry count sits right after the clock: u64 n + n x (u32, u64)
    ck = 8 + 12 * len(states[2][0])
    lying_ne = good[2][:ck] + (1 << 40).to_bytes(8, "little") + good[2][ck + 8:]
    # the first entry's record count (after its u64 member id) far past the frame
    ck3 = 8 + 12 * len(states[3][0])
    lying_n = good[3][:ck3 + 16] + (1 << 40).to_bytes(8, "little") + good[3][ck3 + 24:] if states[3][1] else None
    parts = [good[0], fr_member, fr_actor, truncated, lying_ne] + ([lying_n] if lying_n else []) + [good[3]]
    blob2 = b"".join(parts)
    off2 = np.cumsum([0] + [len(x) for x in parts]).tolist()
    res = wire.orswot_ingest(dev_bytes(blob2), dev_off(off2), ad, md, ctx=octx)
    st = res.status.cpu().tolist()
    assert st[0] == 0 and st[-1] == 0
    assert st[1] == 2 and st[2] == 2               # missing ids: reported, the rest parsed
    assert st[3] & 1 and st[4] & 1                  # truncated, lying entry count
    if lying_n:
        assert st[5] & 1
    ce, ee = to_host(res.clock), to_host(res.entries)
    np.testing.assert_array_equal(ce[0], clock[0])
    np.testing.assert_array_equal(ee[0], entries[0])
    np.testing.assert_array_equal(ce[-1], clock[3])
    np.testing.assert_array_equal(ee[-1], entries[3])
    for i in (1, 2):  # the parsed part of the frames with a missing id
        np.testing.assert_array_equal(ce[i], clock[0])
        np.testing.assert_array_equal(ee[i], entries[0])
