"""GPU: pairwise CvRDT::merge of value-typed Map states (round 6; crdt_map_{counter,orswot,nested}_merge_batch
through map.counter_merge_batch / orswot_merge_batch / nested_merge_batch): self[i].merge(other[i]) for
N pairs at once, against the
oracle's Map.merge (map.rs:140-220) with the value's merge inside — GCounter / PNCounter
(gcounter.rs:44-54, pncounter.rs:70-82), Orswot (orswot.rs:81-149) and the nested Map<K2, MVReg>
(mvreg.rs:112-128).  Pairs are op-replay replicas of one history (concurrent entries, removes seen by
one side only, deferred removes at both levels); plus the deferred-slot edge cases (equal rm clocks
from both sides merging their key sets, survivors past self's Dcap flagged)."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host
from test_gpu_map_nested import _intern, canon, decode_states, nested_states

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import wire  # noqa: E402


def _slots(def_row, def_clock, def_keys, N, A, Kw, Dcap):
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    for j in range(def_row.shape[0]):
        n = int(def_row[j])
        dcl[n, cnt[n]], dks[n, cnt[n]] = def_clock[j], def_keys[j]
        cnt[n] += 1
    return to_dev(dcl), to_dev(dks), torch.from_numpy(cnt).cuda()


def _slot_list(st, n):
    dcl, dks, cnt = to_host(st.def_clock), to_host(st.def_keys), st.def_count.cpu().numpy()
    return [(dcl[n, i], O.bitmap_members(dks[n, i])) for i in range(int(cnt[n]))]


# ---- Map<K, GCounter / PNCounter> -------------------------------------------------------------------
def _counter_frames(maps, K, A, W, Dcap):
    d = O.map_counter_to_dense(maps, K, A, W)
    return wire.MapCounterFrames(to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["val"]),
                                 *_slots(d["def_row"], d["def_clock"], d["def_keys"], len(maps), A, (K + 63) // 64, Dcap))


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("seed,N,K,A", [(1, 12, 5, 4), (2, 20, 9, 7), (3, 8, 70, 5), (4, 10, 6, 70)])
def test_counter_merge_batch(gpu_ctx, W, seed, N, K, A):
    maps = O.map_counter_objects(2 * N, K, A, W, seed=seed, steps=12 * N)
    Dcap = max([len(m.deferred) for m in maps] + [1]) * 2
    me, other = _counter_frames(maps[:N], K, A, W, Dcap), _counter_frames(maps[N:], K, A, W, Dcap)
    status = cg.map.counter_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    c, e, v = to_host(me.clock), to_host(me.ec), to_host(me.val)
    for i in range(N):
        exp = maps[i].copy()
        exp.merge(maps[N + i].copy())
        assert O.dense_to_map_counter(c[i], e[i], v[i], _slot_list(me, i)) == exp, i
    # other is read only
    assert torch.equal(other.clock, _counter_frames(maps[N:], K, A, W, Dcap).clock)


def test_counter_merge_batch_deferred_slots(gpu_ctx):
    """Pair 0: equal rm clocks on both sides -> one survivor with both key sets.  Pair 1: two distinct
    removes from the future with self's Dcap 1 -> status bit 0, the first survivor kept.  Pair 2:
    other's clock dominates self's remove -> dropped, its key's entry forgotten."""
    K, A, W, Dcap = 4, 3, 1, 1
    mk = lambda: O.Map(O.GCounter)  # noqa: E731
    a, b = [mk() for _ in range(3)], [mk() for _ in range(3)]
    a[0].apply(O.MapRm(O.VClock({0: 5}), {0}))
    b[0].apply(O.MapRm(O.VClock({0: 5}), {1}))
    a[1].apply(O.MapRm(O.VClock({1: 4}), {2}))
    b[1].apply(O.MapRm(O.VClock({2: 4}), {3}))
    a[2].apply(O.MapUp(O.Dot(0, 1), 2, O.Dot(0, 1)))
    a[2].apply(O.MapRm(O.VClock({1: 2}), {2}))
    b[2].apply(O.MapUp(O.Dot(1, 1), 3, O.Dot(1, 1)))
    b[2].apply(O.MapUp(O.Dot(1, 2), 3, O.Dot(1, 2)))
    me, other = _counter_frames(a, K, A, W, Dcap), _counter_frames(b, K, A, W, Dcap)
    status = cg.map.counter_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert list(status) == [0, 1, 0], status
    c, e, v = to_host(me.clock), to_host(me.ec), to_host(me.val)
    for i in (0, 2):
        exp = a[i].copy()
        exp.merge(b[i].copy())
        assert O.dense_to_map_counter(c[i], e[i], v[i], _slot_list(me, i)) == exp, i
    assert _slot_list(me, 0)[0][1] == {0, 1}
    assert int(me.def_count[1]) == 1 and list(_slot_list(me, 1)[0][0]) == [0, 4, 0]


def test_counter_merge_batch_validation(gpu_ctx):
    maps = O.map_counter_objects(4, 3, 3, 2, seed=5, steps=20)
    me, other = _counter_frames(maps[:2], 3, 3, 2, 4), _counter_frames(maps[2:], 3, 3, 2, 4)
    with pytest.raises(ValueError):
        cg.map.counter_merge_batch(me, other._replace(ec=other.ec[:, :2].contiguous()), ctx=gpu_ctx)
    bad = other.def_count.clone()
    bad[0] = 5
    before = me.clock.clone()
    with pytest.raises(cg.CrdtGpuError) as ei:  # (the C entry point: EINVAL before anything is written)
        cg.map.counter_merge_batch(me, other._replace(def_count=bad), ctx=gpu_ctx)
    assert ei.value.code == -1 and torch.equal(me.clock, before)
    z = _counter_frames([], 3, 3, 2, 4)
    assert cg.map.counter_merge_batch(z, z, ctx=gpu_ctx).numel() == 0


# ---- Map<K, Orswot<M>> -----------------------------------------------------------------------------
def _orswot_frames(ctx, maps, K, M, A, Dcap):
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
    slots = _slots(d["def_row"], d["def_clock"], d["def_keys"], N, A, (K + 63) // 64, Dcap)
    return wire.MapOrswotFrames(res.clock, res.ec, res.oc, res.ent, res.vd_n, res.vd_clock, res.vd_mem, *slots)


def _orswot_state(st, n, K):
    vn, vc, vm = st.vd_n.cpu().numpy(), to_host(st.vd_clock), to_host(st.vd_mem)
    vd = {k: [(vc[n, k, i], O.bitmap_members(vm[n, k, i:i + 1] if vm.ndim == 3 else vm[n, k, i]))
              for i in range(int(vn[n, k]))] for k in range(K)}
    return O.dense_to_map_orswot(to_host(st.clock)[n], to_host(st.ec)[n], to_host(st.oc)[n], to_host(st.ent)[n], vd,
                                 _slot_list(st, n))


@pytest.mark.parametrize("seed,N,K,M,A", [(1, 10, 4, 6, 4), (2, 16, 6, 9, 6), (3, 8, 3, 70, 5), (4, 8, 5, 8, 70)])
def test_orswot_merge_batch(gpu_ctx, seed, N, K, M, A):
    maps = O.map_orswot_objects(2 * N, K, M, A, seed=seed, steps=10 * N)
    exps = []
    for i in range(N):
        exp = maps[i].copy()
        exp.merge(maps[N + i].copy())
        exps.append(exp)
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in maps + exps for e in x.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    Dcap = max([len(m.deferred) for m in maps] + [1]) * 2
    me, other = _orswot_frames(gpu_ctx, maps[:N], K, M, A, Dcap), _orswot_frames(gpu_ctx, maps[N:], K, M, A, Dcap)
    status = cg.map.orswot_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    for i in range(N):
        got = _orswot_state(me, i, K)
        assert got.clock == exps[i].clock and got.entries == exps[i].entries and got.deferred == exps[i].deferred, i


# ---- Map<K, Map<K2, MVReg<u64>>> ------------------------------------------------------------------
@pytest.mark.parametrize("seed,N,K,K2,A", [(1, 10, 3, 4, 4), (2, 16, 5, 6, 5), (3, 8, 4, 20, 8), (4, 6, 3, 64, 64)])
def test_nested_merge_batch(gpu_ctx, seed, N, K, K2, A):
    maps = O.nested_map_objects(2 * N, K, K2, A, seed=seed, steps=8 * N)
    dense, back, Ad, Kd, Jd = _intern(maps)
    exps = []
    for i in range(N):
        exp = maps[i].copy()
        exp.merge(maps[N + i].copy())
        exps.append(exp)
    Dcap = max([len(m.deferred) for m in maps] + [1]) * 2
    sa, slots_a, _ = nested_states(dense[:N], Kd, Jd, Ad, Dcap)
    sb, slots_b, _ = nested_states(dense[N:], Kd, Jd, Ad, Dcap)
    me, other = wire.MapNestedFrames(*sa, *slots_a), wire.MapNestedFrames(*sb, *slots_b)
    status = cg.map.nested_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    for i in range(N):
        got = back(decode_states(me, i, _slot_list(me, i)))
        assert canon(got) == canon(exps[i]), i


@pytest.mark.parametrize("K2,A,seed", [(200, 6, 5), (256, 70, 6)])
def test_nested_merge_batch_wide_inner_keys(gpu_ctx, K2, A, seed):
    """K2 > 64 (inner key sets of K2w mask words), states not interned so the inner keys spread over
    the whole range."""
    N, K = 6, 3
    maps = O.nested_map_objects(2 * N, K, K2, A, seed=seed, steps=300)
    exps = []
    for i in range(N):
        exp = maps[i].copy()
        exp.merge(maps[N + i].copy())
        exps.append(exp)
    Dcap = max([len(m.deferred) for m in maps] + [1]) * 2
    sa, slots_a, _ = nested_states(maps[:N], K, K2, A, Dcap)
    sb, slots_b, _ = nested_states(maps[N:], K, K2, A, Dcap)
    assert sa.id_keys.dim() == 4
    me, other = wire.MapNestedFrames(*sa, *slots_a), wire.MapNestedFrames(*sb, *slots_b)
    status = cg.map.nested_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    for i in range(N):
        assert canon(decode_states(me, i, _slot_list(me, i))) == canon(exps[i]), i
    assert any(j >= 64 for e in exps[0].entries.values() for j in e.val.entries) or K2 <= 64


def test_counter_merge_batch_different_dcaps(gpu_ctx):
    """self and other with different slot capacities (other's Dcap 3 x self's): the pool takes both."""
    N, K, A, W = 10, 6, 5, 2
    maps = O.map_counter_objects(2 * N, K, A, W, seed=8, steps=20 * N)
    Dc = max([len(m.deferred) for m in maps] + [1])
    me, other = _counter_frames(maps[:N], K, A, W, 2 * Dc), _counter_frames(maps[N:], K, A, W, 3 * Dc)
    status = cg.map.counter_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    c, e, v = to_host(me.clock), to_host(me.ec), to_host(me.val)
    for i in range(N):
        exp = maps[i].copy()
        exp.merge(maps[N + i].copy())
        assert O.dense_to_map_counter(c[i], e[i], v[i], _slot_list(me, i)) == exp, i


def test_orswot_merge_batch_other_untouched_and_validation(gpu_ctx):
    N, K, M, A = 6, 4, 5, 4
    maps = O.map_orswot_objects(2 * N, K, M, A, seed=11, steps=60, p_vrm=0.5)
    me, other = _orswot_frames(gpu_ctx, maps[:N], K, M, A, 8), _orswot_frames(gpu_ctx, maps[N:], K, M, A, 8)
    snap = [t.clone() for t in other]
    bad = other.vd_n.clone()
    bad[0, 0] = 17
    with pytest.raises(cg.CrdtGpuError):
        cg.map.orswot_merge_batch(me, other._replace(vd_n=bad), ctx=gpu_ctx)
    exps = []
    for i in range(N):
        exp = maps[i].copy()
        exp.merge(maps[N + i].copy())
        exps.append(exp)
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in exps for e in x.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    status = cg.map.orswot_merge_batch(me, other, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    for a_, b_ in zip(snap, other):
        assert torch.equal(a_, b_)
    for i in range(N):
        got = _orswot_state(me, i, K)
        assert got.clock == exps[i].clock and got.entries == exps[i].entries and got.deferred == exps[i].deferred, i
