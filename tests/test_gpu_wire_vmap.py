"""GPU: serde wire ingest / egress of the value-typed Maps (round 5; crdt_map_{counter,orswot,nested}_
ingest / _egress) against the oracle's bincode restatement of the derives
(oracle.bc_map_obj / unbc_map_obj; map.rs:31-47 with gcounter.rs:25-28, pncounter.rs:28-32,
orswot.rs:20-25 or Map<K2, MVReg> (mvreg.rs:32-35, the reference's TMap) as the value):
  * ingest of op-replay states (deferred removes at both levels) equals the oracle's dense layouts
    (map_counter_to_dense / map_orswot_to_dense), and egress writes the same frames byte for byte;
  * serialized replicas -> ingest -> CmRDT::apply op streams -> egress -> decode == the oracle's
    Map.apply (map.rs:119-137) of the same ops;
  * truncated frames, ids missing from a dictionary and deferred lists past capacity are reported
    per state."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_host
from test_gpu_wire import actor_dict, dev_bytes, dev_off, host_frames, u64_dict

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import wire  # noqa: E402


def _check_map_deferred(st, d, N):
    dc, dk, cnt = to_host(st.def_clock), to_host(st.def_keys), st.def_count.cpu().numpy()
    rows = d["def_row"].astype(np.int64)
    for n in range(N):
        js = np.flatnonzero(rows == n)
        assert cnt[n] == len(js), n
        np.testing.assert_array_equal(dc[n, :len(js)], d["def_clock"][js])
        np.testing.assert_array_equal(dk[n, :len(js)], d["def_keys"][js])


@pytest.mark.parametrize("W,A", [(1, 6), (2, 6), (1, 70), (2, 130)])
def test_map_counter_ingest_egress(gpu_ctx, W, A):
    N, K = 24, 6
    maps = O.map_counter_objects(N, K, A, W, seed=40 if A <= 6 else 40 + A, steps=220 if A <= 6 else 260)
    rng = np.random.default_rng(W + A)
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)
    blob, off = O.frames([O.bc_map_obj(m, aids, kids) for m in maps])
    Dcap = max(1, max(len(m.deferred) for m in maps))
    st, status = wire.map_counter_ingest(dev_bytes(blob), dev_off(off), ad, kd, W, Dcap, ctx=gpu_ctx)
    assert (status.cpu().numpy() == 0).all()
    d = O.map_counter_to_dense(maps, K, A, W)
    for nm in ("clock", "ec", "val"):
        np.testing.assert_array_equal(to_host(getattr(st, nm)), d[nm], err_msg=nm)
    _check_map_deferred(st, d, N)
    assert d["def_row"].shape[0] > 0
    eoff, edata = wire.map_counter_egress(st, ad, kd, ctx=gpu_ctx)
    assert eoff.cpu().tolist() == off
    assert bytes(edata.cpu().numpy().tobytes()) == blob  # canonical frames round-trip byte for byte


@pytest.mark.parametrize("M,A", [(4, 5), (70, 6), (5, 80)])
def test_map_orswot_ingest_egress(gpu_ctx, M, A):
    N, K = 16, 4
    maps = O.map_orswot_objects(N, K, M, A, seed=60 + M + A, steps=180, p_vrm=0.45)
    if any(len(e.val.deferred) > 16 for m in maps for e in m.entries.values()):
        pytest.skip("nested deferred past the layout's 16 slots")
    rng = np.random.default_rng(M + A)
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)
    mids, md = u64_dict(rng, M)
    blob, off = O.frames([O.bc_map_obj(m, aids, kids, mids) for m in maps])
    Dcap = max(1, max(len(m.deferred) for m in maps))
    st, status = wire.map_orswot_ingest(dev_bytes(blob), dev_off(off), ad, kd, md, Dcap, ctx=gpu_ctx)
    assert (status.cpu().numpy() == 0).all()
    d = O.map_orswot_to_dense(maps, K, M, A)
    for nm in ("clock", "ec", "oc", "ent"):
        np.testing.assert_array_equal(to_host(getattr(st, nm)), d[nm], err_msg=nm)
    vn, vc, vm = st.vd_n.cpu().numpy(), to_host(st.vd_clock), to_host(st.vd_mem)
    vo = d["vd_off"].astype(np.int64)
    for n in range(N):
        for k in range(K):
            a, b = vo[n * K + k], vo[n * K + k + 1]
            assert vn[n, k] == b - a, (n, k)
            np.testing.assert_array_equal(vc[n, k, :b - a], d["vd_clock"][a:b])
            np.testing.assert_array_equal(vm[n, k, :b - a], d["vd_members"][a:b])
    _check_map_deferred(st, d, N)
    assert vo[-1] > 0 and d["def_row"].shape[0] > 0
    eoff, edata = wire.map_orswot_egress(st, ad, kd, md, ctx=gpu_ctx)
    assert eoff.cpu().tolist() == off
    assert bytes(edata.cpu().numpy().tobytes()) == blob


@pytest.mark.parametrize("W", [1, 2])
def test_map_counter_apply_through_bytes(gpu_ctx, W):
    """Serialized replicas -> ingest -> counter_apply_batch -> egress -> decode == Map.apply."""
    from test_gpu_map_counter_apply import _streams
    N, K, A, T, Dcap = 24, 6, 6, 40, 16
    maps = O.map_counter_objects(N, K, A, W, seed=40, steps=220)
    rng = np.random.default_rng(70 + W)
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)
    blob, off = O.frames([O.bc_map_obj(m, aids, kids) for m in maps])
    st, status = wire.map_counter_ingest(dev_bytes(blob), dev_off(off), ad, kd, W, Dcap, ctx=gpu_ctx)
    assert (status.cpu().numpy() == 0).all()
    streams, oops = _streams(rng, maps, K, A, W, T)
    ops = cg.map.encode_counter_ops(streams, A, "cuda:0")
    ast = cg.map.counter_apply_batch(st.clock, st.ec, st.val, st.def_clock, st.def_keys, st.def_count, ops,
                                     ctx=gpu_ctx).cpu().numpy()
    assert (ast == 0).all(), ast
    eoff, edata = wire.map_counter_egress(st, ad, kd, ctx=gpu_ctx)
    vnew = O.GCounter if W == 1 else O.PNCounter
    deferred = 0
    for n, fr in enumerate(host_frames(edata, eoff)):
        got, pos = O.unbc_map_obj(fr, vnew, aids, kids)
        assert pos == len(fr)
        exp = maps[n].copy()
        for op in oops[n]:
            exp.apply(op)
        assert got == exp, n
        deferred += len(exp.deferred)
    assert deferred > 0


def test_map_orswot_apply_through_bytes(gpu_ctx):
    """Serialized replicas -> ingest -> orswot_apply_batch -> egress -> decode == Map.apply with the
    nested Orswot ops (deferred removes at both levels)."""
    from test_gpu_map_orswot_apply import _streams
    N, K, M, A, T, Dcap = 16, 4, 6, 5, 30, 16
    maps = O.map_orswot_objects(N, K, M, A, seed=64, steps=160, p_vrm=0.4)
    rng = np.random.default_rng(71)
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)
    mids, md = u64_dict(rng, M)
    blob, off = O.frames([O.bc_map_obj(m, aids, kids, mids) for m in maps])
    st, status = wire.map_orswot_ingest(dev_bytes(blob), dev_off(off), ad, kd, md, Dcap, ctx=gpu_ctx)
    assert (status.cpu().numpy() == 0).all()
    exps = [m.copy() for m in maps]
    streams, oops = _streams(rng, exps, K, M, A, T)
    for n in range(N):
        for op in oops[n]:
            exps[n].apply(op)
    if any(len(e.val.deferred) > 16 for x in exps for e in x.entries.values()) or \
            any(len(x.deferred) > Dcap for x in exps):
        pytest.skip("past the kernel's deferred capacity")
    ops = cg.map.encode_orswot_map_ops(streams, A, "cuda:0")
    ast = cg.map.orswot_apply_batch(st, st.def_clock, st.def_keys, st.def_count, ops, ctx=gpu_ctx).cpu().numpy()
    assert (ast == 0).all(), ast
    eoff, edata = wire.map_orswot_egress(st, ad, kd, md, ctx=gpu_ctx)
    nested = 0
    for n, fr in enumerate(host_frames(edata, eoff)):
        got, pos = O.unbc_map_obj(fr, O.Orswot, aids, kids, mids)
        assert pos == len(fr)
        assert got.clock == exps[n].clock and got.entries == exps[n].entries, n
        assert got.deferred == exps[n].deferred, n
        nested += sum(len(e.val.deferred) for e in exps[n].entries.values())
    assert nested > 0


def test_value_map_malformed_missing_and_capacity(gpu_ctx):
    """Status bits per state: 1 = malformed (truncated / trailing bytes), 2 = an id missing from a
    dictionary (skipped), 4 = more removes than the slots (the excess dropped)."""
    rng = np.random.default_rng(72)
    A, K, M = 3, 4, 4
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)
    mids, md = u64_dict(rng, M)
    m = O.Map(O.PNCounter)
    m.clock = O.VClock({0: 2, 1: 1})
    v = O.PNCounter()
    v.p.inner = O.VClock({0: 2})
    m.entries[1] = O.MapEntry(O.VClock({0: 2}), v)
    good = O.bc_map_obj(m, aids, kids)
    m2 = m.copy()
    for i in range(3):
        m2.deferred[O.VClock({2: 5 + i})] = {i}
    over = O.bc_map_obj(m2, aids, kids)
    missing = O.bc_map_obj(m, aids, [kids[0], kids[1] + 1 if kids[1] + 1 not in kids else kids[1] - 1] + list(kids[2:]))
    blob, off = O.frames([good, good[:-4], good + b"\0\0\0\0", over, missing])
    st, status = wire.map_counter_ingest(dev_bytes(blob), dev_off(off), ad, kd, 2, 2, ctx=gpu_ctx)
    s = status.cpu().numpy()
    assert s[0] == 0 and s[1] & wire.BAD and s[2] & wire.BAD and s[3] == wire.CAP and s[4] == wire.MISSING, s
    assert int(st.def_count[3]) == 2
    # Orswot: a nested list past 16 and an unknown member
    o = O.Map(O.Orswot)
    o.clock = O.VClock({0: 3})
    ov = O.Orswot()
    ov.clock = O.VClock({0: 3})
    ov.entries[2] = O.VClock({0: 3})
    for i in range(17):
        ov.deferred[O.VClock({1: 10 + i})] = {i % M}
    o.entries[0] = O.MapEntry(O.VClock({0: 3}), ov)
    many = O.bc_map_obj(o, aids, kids, mids)
    o2 = O.Map(O.Orswot)
    o2.clock = O.VClock({0: 1})
    ov2 = O.Orswot()
    ov2.clock = O.VClock({0: 1})
    ov2.entries[1] = O.VClock({0: 1})
    o2.entries[2] = O.MapEntry(O.VClock({0: 1}), ov2)
    bad_mids = np.array([mids[0], mids[1] ^ 1 if (mids[1] ^ 1) not in mids else mids[1] + 7, mids[2], mids[3]],
                        np.uint64)
    unknown = O.bc_map_obj(o2, aids, kids, bad_mids)
    blob, off = O.frames([many, unknown, many[:-8]])
    ost, status = wire.map_orswot_ingest(dev_bytes(blob), dev_off(off), ad, kd, md, 1, ctx=gpu_ctx)
    s = status.cpu().numpy()
    assert s[0] == wire.CAP and s[1] == wire.MISSING and s[2] & wire.BAD, s
    assert int(ost.vd_n[0, 0]) == 16
    assert to_host(ost.ec)[1, 2].any() and not to_host(ost.ent)[1, 2].any()  # the unknown member skipped


def _nested_fits(m):
    return (len(m.deferred) <= 16 and all(len(e.val.deferred) <= 16 for e in m.entries.values())
            and all(len(ie.val.vals) <= 8 for e in m.entries.values() for ie in e.val.entries.values()))


@pytest.mark.parametrize("K2,A", [(6, 5), (64, 4), (5, 70), (200, 5), (256, 6)])  # (K2 > 64: K2w key-set words)
def test_map_nested_ingest_egress(gpu_ctx, K2, A):
    """Map<u32, Map<u32, MVReg<u64>>> (test/map.rs:10): ingest equals the state layout built from the
    oracle objects, egress reproduces the frames byte for byte."""
    from test_gpu_map_nested import nested_states
    K = 4
    maps = [m for m in O.nested_map_objects(28, K, K2, A, seed=50 + K2 + A, steps=200, p_irm=0.5, p_ooo=0.8,
                                            p_rm=0.3) if _nested_fits(m)]
    N = len(maps)
    rng = np.random.default_rng(K2 + A)
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)
    iids, idd = actor_dict(rng, K2)
    blob, off = O.frames([O.bc_map_obj(m, aids, kids, iid=iids) for m in maps])
    Dcap = 16
    st, status = wire.map_nested_ingest(dev_bytes(blob), dev_off(off), ad, kd, idd, Dcap, ctx=gpu_ctx)
    assert (status.cpu().numpy() == 0).all()
    exp, slots, _ = nested_states(maps, K, K2, A)
    for nm in exp._fields:
        np.testing.assert_array_equal(getattr(st, nm).cpu().numpy(), getattr(exp, nm).cpu().numpy(), err_msg=nm)
    for got, e in zip((st.def_clock, st.def_keys, st.def_count), slots):
        np.testing.assert_array_equal(got.cpu().numpy(), e.cpu().numpy())
    assert int(st.id_n.sum()) > 0 and int(st.def_count.sum()) > 0
    eoff, edata = wire.map_nested_egress(st, ad, kd, idd, ctx=gpu_ctx)
    assert eoff.cpu().tolist() == off
    assert bytes(edata.cpu().numpy().tobytes()) == blob


def test_map_nested_apply_through_bytes(gpu_ctx):
    """Serialized TMap replicas -> ingest -> nested_apply_batch -> egress -> decode == Map.apply."""
    from test_gpu_map_nested import canon
    from test_gpu_map_nested_apply import _regs_in_order, _streams
    K, K2, A, T = 4, 6, 5, 30
    maps = [m for m in O.nested_map_objects(32, K, K2, A, seed=81, steps=200, p_irm=0.5, p_ooo=0.8, p_rm=0.3)
            if _nested_fits(m)][:24]
    rng = np.random.default_rng(73)
    streams, oops = _streams(rng, maps, K, K2, A, T)
    exps = [m.copy() for m in maps]
    for n, e in enumerate(exps):
        for op in oops[n]:
            e.apply(op)
    keep = [n for n, e in enumerate(exps) if _nested_fits(e)]
    maps, exps, streams = [maps[n] for n in keep], [exps[n] for n in keep], [streams[n] for n in keep]
    aids, ad = actor_dict(rng, A)
    kids, kd = actor_dict(rng, K)
    iids, idd = actor_dict(rng, K2)
    blob, off = O.frames([O.bc_map_obj(m, aids, kids, iid=iids) for m in maps])
    st, status = wire.map_nested_ingest(dev_bytes(blob), dev_off(off), ad, kd, idd, 16, ctx=gpu_ctx)
    assert (status.cpu().numpy() == 0).all()
    ops = cg.map.encode_nested_ops(streams, A, "cuda:0")
    ast = cg.map.nested_apply_batch(st, st.def_clock, st.def_keys, st.def_count, ops, ctx=gpu_ctx).cpu().numpy()
    assert (ast == 0).all(), ast
    eoff, edata = wire.map_nested_egress(st, ad, kd, idd, ctx=gpu_ctx)
    for n, fr in enumerate(host_frames(edata, eoff)):
        got, pos = O.unbc_map_obj(fr, "nested", aids, kids, iid=iids)
        assert pos == len(fr)
        assert canon(got) == canon(exps[n]) and _regs_in_order(got) == _regs_in_order(exps[n]), n
    assert len(exps) >= 12
