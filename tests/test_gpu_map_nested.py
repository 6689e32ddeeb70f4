"""GPU parity: Map<K, Map<K2, MVReg<u64>>> lub_many (crdt_map_nested_lub_many, round 5) — the nested
type of the reference's own Map tests (TMap, /root/reference/test/map.rs:10; TestMap, src/map.rs:359).

Every merge of the reference's TMap tests runs on the GPU here: `gpu_merge(a, b)` interns the two
states' actors / keys to dense indices, folds [a, b] with the kernel (Map::new().merge(a).merge(b) ==
a.merge(b) for the reference's states) and turns the result back into oracle objects, so the
reference's own assertions check the kernel:
  test/map.rs:148-174 (reset-remove), :197-235 (add bias), :331-362, :364-404, :406-430, :432-478,
  :480-516 (the quickcheck regressions) and the merge laws of :524-827 (commutative, associative,
  idempotent, merge-followed-by-merge, op exchange == merge) over seeded quickcheck-style ops.
Plus op-replay histories (inner writes and inner removes read at replicas that have seen more, so
removes defer at both levels) folded over many replicas against the oracle's left fold."""
import random
from typing import NamedTuple

import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host
from oracle import Dot, Map, MapRm, MapUp, MVReg, MVRegPut, VClock

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def TMap():  # test/map.rs:9
    return Map(lambda: Map(MVReg))


def vc(*dots):
    return VClock.from_dots(Dot(a, c) for a, c in dots)


def apply_ops(m, ops):  # test/map.rs:473-477
    for op in ops:
        m.apply(op)


def build_ops(actor, ops_data):  # test/map.rs:11-46
    ops = []
    for i, (choice, inner_choice, key, inner_key, val) in enumerate(ops_data):
        clock = vc((actor, i))
        if choice % 2 == 0:
            if inner_choice % 2 == 0:
                inner = MapUp(clock.inc(actor), inner_key, MVRegPut(clock.copy(), val))
            else:
                inner = MapRm(clock.copy(), {inner_key})
            ops.append(MapUp(clock.inc(actor), key, inner))
        else:
            ops.append(MapRm(clock.copy(), {key}))
    return actor, ops


# ---- dense interning of reference-shaped states ----------------------------------------------------
class _Dict:
    def __init__(self, items):
        self.fwd = {x: i for i, x in enumerate(sorted(items))}
        self.inv = {i: x for x, i in self.fwd.items()}


def _clocks(m):
    yield m.clock
    for rm in m.deferred:
        yield rm
    for e in m.entries.values():
        yield e.clock
        yield e.val.clock
        for rm in e.val.deferred:
            yield rm
        for ie in e.val.entries.values():
            yield ie.clock
            for c, _ in ie.val.vals:
                yield c


def _map_clock(c, d):
    return VClock({d[a]: n for a, n in c.dots.items()})


def _intern(maps, extra=None, with_dicts=False):
    acts, keys, ikeys = (set(x) for x in extra) if extra else (set(), set(), set())
    for m in maps:
        for c in _clocks(m):
            acts |= set(c.dots)
        keys |= set(m.entries)
        for ks in m.deferred.values():
            keys |= set(ks)
        for e in m.entries.values():
            ikeys |= set(e.val.entries)
            for ks in e.val.deferred.values():
                ikeys |= set(ks)
    A, K, J = _Dict(acts or {0}), _Dict(keys or {0}), _Dict(ikeys or {0})

    def conv(m, a, k, j):
        n = TMap()
        n.clock = _map_clock(m.clock, a)
        for rm, ks in m.deferred.items():
            n.deferred[_map_clock(rm, a)] = {k[x] for x in ks}
        for key, e in m.entries.items():
            inner = Map(MVReg)
            inner.clock = _map_clock(e.val.clock, a)
            for rm, ks in e.val.deferred.items():
                inner.deferred[_map_clock(rm, a)] = {j[x] for x in ks}
            for ik, ie in e.val.entries.items():
                inner.entries[j[ik]] = O.MapEntry(_map_clock(ie.clock, a),
                                                  MVReg([(_map_clock(c, a), v) for c, v in ie.val.vals]))
            n.entries[k[key]] = O.MapEntry(_map_clock(e.clock, a), inner)
        return n

    dense = [conv(m, A.fwd, K.fwd, J.fwd) for m in maps]
    back = lambda m: conv(m, A.inv, K.inv, J.inv)  # noqa: E731
    if with_dicts:
        return dense, back, A, K, J
    return dense, back, len(A.fwd), len(K.fwd), len(J.fwd)


def gpu_fold(ctx, maps):
    """acc = Map::new(); for m in maps: acc.merge(m), every merge on the GPU (one nested_lub_many)."""
    dense, back, A, K, K2 = _intern(maps)
    if A > 256 or K2 > 256:
        pytest.skip("more than 256 actors / inner keys in one case")
    V = max([len(ie.val.vals) for m in dense for e in m.entries.values() for ie in e.val.entries.values()] + [1])
    d = O.nested_map_to_dense(dense, K, K2, A, V)
    D = d["def_row"].shape[0]
    kw = {}
    if D:
        kw = dict(def_off=[0, D], def_row=torch.from_numpy(d["def_row"].astype(np.int32)).cuda(),
                  def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"]))
    Di = d["id_clock"].shape[0]
    ikw = dict(id_clock=to_dev(d["id_clock"]), id_keys=to_dev(d["id_keys"])) if Di else {}
    res = cg.map.nested_lub_many(to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["ic"]), to_dev(d["iec"]),
                                 to_dev(d["ivc"]), to_dev(d["ivv"]), to_dev(d["id_off"]), ctx=ctx, **ikw, **kw)
    dset = []
    if D:
        dset = [(np.array(rm, np.uint64), ks)
                for rm, ks in cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys)]
    idn = res.id_n.cpu().numpy()
    idc, idk = to_host(res.id_clock), to_host(res.id_keys)
    ideferred = {k: [(idc[k, i], O.bitmap_members(_kw(idk, k, i))) for i in range(int(idn[k]))] for k in range(K)}
    got = O.dense_to_nested_map(to_host(res.clock), to_host(res.ec), to_host(res.ic), to_host(res.iec),
                                to_host(res.ivc), to_host(res.ivv), res.nval.cpu().numpy(), ideferred, dset)
    return back(got)


class _States(NamedTuple):
    """The crdt_map_nested_states layout of N states (nested_lub_many's output shapes, G = N)."""
    clock: torch.Tensor
    ec: torch.Tensor
    ic: torch.Tensor
    iec: torch.Tensor
    ivc: torch.Tensor
    ivv: torch.Tensor
    nval: torch.Tensor
    id_n: torch.Tensor
    id_clock: torch.Tensor
    id_keys: torch.Tensor


def nested_states(maps, K, K2, A, Dcap=16, Id=16):
    """Dense objects -> (_States on the device, outer deferred as slots (N, Dcap, A) / (N, Dcap, Kw) /
    (N,) int32, and as a pool (def_clock (D, A), def_state (D,))); Id inner deferred slots per key."""
    N = len(maps)
    d = O.nested_map_to_dense(maps, K, K2, A, 8)
    nval = np.zeros((N, K, K2), np.int32)
    for n, m in enumerate(maps):
        for k, e in m.entries.items():
            for j, ie in e.val.entries.items():
                nval[n, k, j] = len(ie.val.vals)
    idn = np.zeros((N, K), np.int32)
    idc = np.zeros((N, K, Id, A), np.uint64)
    K2w = (K2 + 63) // 64 if K2 > 64 else 1  # inner key sets: K2w mask words past 64 keys
    idk = np.zeros((N, K, Id) if K2w == 1 else (N, K, Id, K2w), np.uint64)
    off = d["id_off"].astype(np.int64)
    for i in range(N * K):
        a, b = off[i], off[i + 1]
        assert b - a <= Id
        idn[i // K, i % K] = b - a
        idc[i // K, i % K, :b - a] = d["id_clock"][a:b]
        idk[i // K, i % K, :b - a] = d["id_keys"][a:b]
    st = _States(to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["ic"]), to_dev(d["iec"]), to_dev(d["ivc"]),
                 to_dev(d["ivv"]), torch.from_numpy(nval).cuda(), torch.from_numpy(idn).cuda(), to_dev(idc),
                 to_dev(idk))
    Kw = (K + 63) // 64
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    for j in range(d["def_row"].shape[0]):
        n = int(d["def_row"][j])
        assert cnt[n] < Dcap
        dcl[n, cnt[n]], dks[n, cnt[n]] = d["def_clock"][j], d["def_keys"][j]
        cnt[n] += 1
    return st, (to_dev(dcl), to_dev(dks), torch.from_numpy(cnt).cuda()), d


def _kw(idk, k, i):
    """Inner-key mask words of held remove i of key k: (K, 16) one word, (K, 16, K2w) past 64 keys."""
    return idk[k, i:i + 1] if idk.ndim == 2 else idk[k, i]


def decode_states(st, n, dfr):
    idn = st.id_n.cpu().numpy()[n]
    idc, idk = to_host(st.id_clock)[n], to_host(st.id_keys)[n]
    K = idn.shape[0]
    idef = {k: [(idc[k, i], O.bitmap_members(_kw(idk, k, i))) for i in range(int(idn[k]))] for k in range(K)}
    return O.dense_to_nested_map(to_host(st.clock)[n], to_host(st.ec)[n], to_host(st.ic)[n], to_host(st.iec)[n],
                                 to_host(st.ivc)[n], to_host(st.ivv)[n], st.nval.cpu().numpy()[n], idef, dfr)


def _slot_deferred(slots, n):
    dcl, dks, cnt = to_host(slots[0]), to_host(slots[1]), slots[2].cpu().numpy()
    return [(dcl[n, i], O.bitmap_members(dks[n, i])) for i in range(int(cnt[n]))]


def _op_ids(ops):
    acts, keys, ikeys, clocks = set(), set(), set(), []
    for op in ops:
        if isinstance(op, MapRm):
            clocks.append(op.clock)
            keys |= set(op.keyset)
            continue
        acts.add(op.dot.actor)
        keys.add(op.key)
        if isinstance(op.op, MapRm):
            clocks.append(op.op.clock)
            ikeys |= set(op.op.keyset)
        else:
            acts.add(op.op.dot.actor)
            ikeys.add(op.op.key)
            clocks.append(op.op.op.clock)
    for c in clocks:
        acts |= set(c.dots)
    return acts, keys, ikeys


def _map_vals(m, f):
    n = m.copy()
    for e in n.entries.values():
        for ie in e.val.entries.values():
            ie.val.vals = [(c, f[v]) for c, v in ie.val.vals]
    return n


def gpu_apply(ctx, m, ops):
    """for op in ops: m.apply(op), every apply on the GPU (one crdt_map_nested_apply_batch stream);
    returns the new state.  Register values that are not u64 travel as ids (MVReg compares clocks only)."""
    vals = {v for e in m.entries.values() for ie in e.val.entries.values() for _, v in ie.val.vals}
    vals |= {op.op.op.val for op in ops if isinstance(op, MapUp) and isinstance(op.op, MapUp)}
    if not all(isinstance(v, int) and 0 <= v < 2**64 for v in vals):
        fv = {v: i for i, v in enumerate(sorted(vals, key=repr))}
        inv = {i: v for v, i in fv.items()}
        ops = [MapUp(op.dot, op.key, MapUp(op.op.dot, op.op.key, MVRegPut(op.op.op.clock, fv[op.op.op.val])))
               if isinstance(op, MapUp) and isinstance(op.op, MapUp) else op for op in ops]
        return _map_vals(gpu_apply(ctx, _map_vals(m, fv), ops), inv)
    dense, back, Ad, Kd, Jd = _intern([m], extra=_op_ids(ops), with_dicts=True)
    A, K, K2 = len(Ad.fwd), len(Kd.fwd), len(Jd.fwd)
    if A > 512 or K2 > 256:
        pytest.skip("more than 512 actors / 256 inner keys in one case")
    st, slots, _ = nested_states(dense, K, K2, A)
    row = lambda c: {Ad.fwd[a]: n for a, n in c.dots.items()}  # noqa: E731
    stream = []
    for op in ops:
        if isinstance(op, MapRm):
            stream.append(("rm", row(op.clock), [Kd.fwd[k] for k in op.keyset]))
        elif isinstance(op.op, MapRm):
            stream.append(("irm", Ad.fwd[op.dot.actor], op.dot.counter, Kd.fwd[op.key], row(op.op.clock),
                           [Jd.fwd[j] for j in op.op.keyset]))
        else:
            put = op.op.op
            stream.append(("put", Ad.fwd[op.dot.actor], op.dot.counter, Kd.fwd[op.key], Ad.fwd[op.op.dot.actor],
                           op.op.dot.counter, Jd.fwd[op.op.key], row(put.clock), int(put.val)))
    enc = cg.map.encode_nested_ops([stream], A, "cuda:0", K2=K2)
    status = cg.map.nested_apply_batch(st, *slots, enc, ctx=ctx).cpu().numpy()
    assert status[0] == 0, status
    return back(decode_states(st, 0, _slot_deferred(slots, 0)))


def gpu_forget(ctx, m, clock):
    """m.forget(clock) on the GPU (crdt_map_nested_forget_batch); returns the new state."""
    dense, back, Ad, Kd, Jd = _intern([m], extra=(set(clock.dots), set(), set()), with_dicts=True)
    A, K, K2 = len(Ad.fwd), len(Kd.fwd), len(Jd.fwd)
    if A > 512 or K2 > 256:
        pytest.skip("more than 512 actors / 256 inner keys in one case")
    st, _, d = nested_states(dense, K, K2, A)
    y = np.zeros(A, np.uint64)
    for a, c in clock.dots.items():
        y[Ad.fwd[a]] = c
    D = d["def_row"].shape[0]
    dcl = to_dev(d["def_clock"]) if D else None
    dst = torch.from_numpy(d["def_row"].astype(np.int32)).cuda() if D else None
    keep = cg.map.nested_forget_batch(st, to_dev(y), def_clock=dcl, def_state=dst, ctx=ctx)
    dfr = []
    if D:
        kp, hc = keep.cpu().numpy(), to_host(dcl)
        dfr = [(hc[j], O.bitmap_members(d["def_keys"][j])) for j in range(D) if kp[j]]
    return back(decode_states(st, 0, dfr))


@pytest.fixture
def gm(gpu_ctx):
    def merge(a, b):  # a.merge(b) on the GPU; returns the merged state
        return gpu_fold(gpu_ctx, [a, b])
    return merge


def canon(m):
    """A comparable form of a nested Map state with each MVReg's values as a sorted multiset: op-replay
    histories can leave one (clock, value) twice in a register (the oracle's fold — a restatement of
    mvreg.rs:112-128 — does so too), where MVReg's own PartialEq (mvreg.rs:62-86) would assert."""
    def c(vc):
        return tuple(sorted(vc.dots.items()))

    def reg(r):
        return tuple(sorted((c(x), v) for x, v in r.vals))

    def inner(n):
        return (c(n.clock), tuple(sorted((j, c(e.clock), reg(e.val)) for j, e in n.entries.items())),
                tuple(sorted((c(rm), tuple(sorted(ks))) for rm, ks in n.deferred.items())))
    return (c(m.clock), tuple(sorted((k, c(e.clock), inner(e.val)) for k, e in m.entries.items())),
            tuple(sorted((c(rm), tuple(sorted(ks))) for rm, ks in m.deferred.items())))


def read_nested(m, k1, k2):
    v = m.get(k1).val
    if v is None:
        return None
    r = v.get(k2).val
    return None if r is None else r.read().val


# ---- the reference's TMap tests, every merge on the GPU --------------------------------------------
def test_reset_remove_semantics(gm):  # test/map.rs:148-174
    m1 = TMap()
    m1.apply(m1.update(101, m1.get(101).derive_add_ctx(74),
                       lambda mp, c: mp.update(110, c, lambda r, c2: r.write(32, c2))))
    m2 = m1.copy()
    m1.apply(m1.rm(101, m1.get(101).derive_rm_ctx()))
    m2.apply(m2.update(101, m2.get(101).derive_add_ctx(37),
                       lambda mp, c: mp.update(220, c, lambda r, c2: r.write(5, c2))))
    snap = m1.copy()
    m1 = gm(m1, m2)
    m2 = gm(m2, snap)
    assert m1 == m2
    inner = m1.get(101).val
    assert inner.get(220).val.read().val == [5]
    assert inner.get(110).val is None
    assert inner.len().val == 1


def test_concurrent_update_and_remove_add_bias(gm):  # test/map.rs:197-235
    m1, m2 = TMap(), TMap()
    op1 = MapRm(vc((1, 1)), {102})
    op2 = m2.update(102, m2.get(102).derive_add_ctx(2),
                    lambda mp, c: mp.update(42, c, lambda r, c2: r.write(7, c2)))
    m1.apply(op1)
    m2.apply(op2)
    m1c = gm(m1, m2)
    m2c = gm(m2, m1)
    m1.apply(op2)
    m2.apply(op1)
    assert m1c == m2c
    assert m1 == m2
    assert m1 == m1c
    assert read_nested(m1c, 102, 42) == [7]


def test_commute_quickcheck_bug(gm):  # test/map.rs:331-362
    ops = [MapRm(vc((45, 1)), {0}),
           MapUp(Dot(45, 2), 0, MapUp(Dot(45, 1), 0, MVRegPut(VClock(), 0)))]
    m = TMap()
    apply_ops(m, ops)
    empty = TMap()
    assert gm(m, empty) == gm(empty, m)


def test_idempotent_quickcheck_bug1(gm):  # test/map.rs:364-404
    ops = [MapUp(Dot(21, 5), 0, MapUp(Dot(21, 1), 32, MVRegPut(VClock(), 42))),
           MapRm(vc((21, 5)), {0}),
           MapUp(Dot(21, 6), 1, MapUp(Dot(21, 1), 0, MVRegPut(VClock(), 0)))]
    m = TMap()
    apply_ops(m, ops)
    assert gm(m, m.copy()) == m


def test_idempotent_quickcheck_bug2(gm):  # test/map.rs:406-430
    m = TMap()
    m.apply(MapUp(Dot(32, 5), 0, MapUp(Dot(32, 5), 0, MVRegPut(VClock(), 0))))
    assert gm(m, m.copy()) == m


def test_op_exchange_same_as_merge_quickcheck1(gm):  # test/map.rs:432-478
    op1 = MapUp(Dot(38, 4), 216, MapUp(Dot(38, 1), 37, MVRegPut(vc((38, 1)), 94)))
    op2 = MapUp(Dot(91, 9), 216, MapUp(Dot(91, 1), 37, MVRegPut(vc((91, 1)), 94)))
    m1, m2 = TMap(), TMap()
    m1.apply(op1)
    m2.apply(op2)
    m1m = gm(m1, m2)
    m2m = gm(m2, m1)
    m1.apply(op2)
    m2.apply(op1)
    assert m1 == m2
    assert m1m == m2m
    assert m1 == m1m and m2 == m2m and m1 == m2m and m2 == m1m
    assert sorted(read_nested(m1m, 216, 37)) == [94, 94]


def test_idempotent_quickcheck1(gm):  # test/map.rs:480-516
    ops = [MapUp(Dot(62, 9), 47, MapUp(Dot(62, 1), 65, MVRegPut(vc((62, 1)), 240))),
           MapUp(Dot(62, 11), 60, MapUp(Dot(62, 1), 193, MVRegPut(vc((62, 1)), 28)))]
    m = TMap()
    apply_ops(m, ops)
    assert gm(m, m.copy()) == m


# ---- quickcheck properties of test/map.rs (seeded), every merge on the GPU --------------------------
def _prim(rng, n_max=40):
    actor = rng.randrange(256)
    ops = [tuple(rng.randrange(256) for _ in range(5)) for _ in range(rng.randrange(n_max))]
    if rng.random() < 0.5:  # quickcheck's u8 generator favours small values: mix both regimes for keys
        ops = [(c, ic, k % 4, ik % 4, v) for c, ic, k, ik, v in ops]
    return actor, ops


def _maps(rng, n):
    while True:
        prims = [_prim(rng) for _ in range(n)]
        if len(set(p[0] for p in prims)) == n:  # the props discard equal actors
            return [build_ops(*p)[1] for p in prims]


@pytest.mark.parametrize("seed", range(24))
def test_prop_map_merge_laws_on_gpu(gm, seed):
    """prop_op_exchange_same_as_merge, prop_merge_commutative, prop_merge_associative,
    prop_merge_followed_by_merge, prop_merge_idempotent (test/map.rs:526-550, :694-721, :660-692,
    :723-748, :750-764), and each GPU merge equal to the oracle's."""
    rng = random.Random(seed)
    ops1, ops2, ops3 = _maps(rng, 3)
    m1, m2, m3 = TMap(), TMap(), TMap()
    apply_ops(m1, ops1)
    apply_ops(m2, ops2)
    apply_ops(m3, ops3)
    for m in (m1, m2):
        assert gm(m, m.copy()) == m  # idempotent
    mm = gm(m1, m2)
    exp = m1.copy()
    exp.merge(m2.copy())
    assert mm == exp  # the oracle's merge
    a, b = m1.copy(), m2.copy()
    apply_ops(a, ops2)
    apply_ops(b, ops1)
    assert a == mm and b == mm  # op exchange == merge
    assert gm(m2, m1) == mm  # commutative
    x = gm(m1, m2)
    y = gm(m2, x)
    assert x == y  # merge followed by merge
    left = gm(gm(m1, m2), m3)
    right = gm(m1, gm(m2, m3))
    assert left == right  # associative


def _wide_ops(rng, actors):
    """One state's op list from many actors (each a quickcheck prim with its own u8 actor): applying the
    concatenation is the merge of the actors' maps (op exchange, test/map.rs:526-550)."""
    ops = []
    for actor in actors:
        _, o = _prim(rng, n_max=8)
        # outer keys over the whole u8 range (few inner removes deferred per key: the fold holds 16), inner
        # keys too (round 6: up to 256 inner keys, their sets as 4 mask words)
        o = [(c, ic, (k * 37 + actor) % 256, ik, v) for c, ic, k, ik, v in o]
        ops.extend(build_ops(actor, o)[1])
    return ops


@pytest.mark.parametrize("seed", range(6))
def test_prop_map_merge_laws_wide_actors_on_gpu(gm, seed):
    """The merge laws of test/map.rs:524-827 on TMap states written by up to 256 distinct u8 actors over
    inner keys from the whole u8 range (the type's whole domain; round 6: the fold takes A <= 256 with
    lane l holding actors l + 64 j, and K2 <= 256 with inner key sets as 4 mask words): three states from
    disjoint actor sets of 60-90 actors each, every merge on the GPU and equal to the oracle's."""
    rng = random.Random(1000 + seed)
    pool = list(range(256))
    rng.shuffle(pool)
    n = [rng.randrange(60, 90) for _ in range(3)]
    groups = [pool[:n[0]], pool[n[0]:n[0] + n[1]], pool[n[0] + n[1]:n[0] + n[1] + n[2]]]
    ops1, ops2, ops3 = (_wide_ops(rng, g) for g in groups)
    m1, m2, m3 = TMap(), TMap(), TMap()
    apply_ops(m1, ops1)
    apply_ops(m2, ops2)
    apply_ops(m3, ops3)
    mm = gm(m1, m2)
    exp = m1.copy()
    exp.merge(m2.copy())
    assert canon(mm) == canon(exp)  # the oracle's merge (> 64 actors: the wide fold)
    assert canon(gm(m1, m1.copy())) == canon(m1)  # idempotent
    a = m1.copy()
    apply_ops(a, ops2)
    assert canon(a) == canon(mm)  # op exchange == merge
    assert canon(gm(m2, m1)) == canon(mm)  # commutative
    assert canon(gm(m2, mm)) == canon(mm)  # merge followed by merge
    left = gm(gm(m1, m2), m3)
    right = gm(m1, gm(m2, m3))
    assert canon(left) == canon(right)  # associative


# ---- op-replay folds over many replicas against the oracle's left fold -------------------------------
@pytest.mark.parametrize("mode", ["", "nmlds=0"])
@pytest.mark.parametrize("seed,R,K,K2,A", [(1, 30, 3, 4, 4), (2, 50, 5, 6, 5), (3, 40, 2, 3, 3),
                                            (4, 70, 6, 8, 6), (5, 25, 4, 20, 8), (6, 40, 3, 64, 64),
                                            (7, 40, 3, 6, 100), (8, 24, 2, 5, 200), (9, 30, 2, 8, 256),
                                            (10, 30, 2, 100, 6), (11, 24, 2, 256, 5), (12, 20, 2, 130, 100)])
def test_map_nested_op_replay_fold(gpu_ctx, seed, R, K, K2, A, mode):
    """Both state placements: the key's inner Map and the staged replica rows in LDS (default, where
    they fit; at K2 = 64, A = 64 they do not) and the inner Map in the key's output rows."""
    gpu_ctx.tune(mode)
    try:
        maps = O.nested_map_objects(R, K, K2, A, seed=seed, steps=8 * R)
        exp = O.map_fold_objects(maps)
        got = gpu_fold(gpu_ctx, maps)
    finally:
        gpu_ctx.tune("nmlds=1")  # (tune specs are additive: restore the default)
    assert canon(got) == canon(exp)


def test_map_nested_deferred_at_both_levels(gpu_ctx):
    """Enough histories that some folds end with inner and outer deferred removes."""
    n_in = n_out = 0
    for seed in range(30, 40):
        maps = O.nested_map_objects(24, 3, 5, 4, seed=seed, steps=220, p_irm=0.5, p_ooo=0.8, p_rm=0.3)
        exp = O.map_fold_objects(maps)
        n_in += sum(len(e.val.deferred) for e in exp.entries.values())
        n_out += len(exp.deferred)
        assert canon(gpu_fold(gpu_ctx, maps)) == canon(exp)
    assert n_in > 0 and n_out > 0


def test_map_nested_groups_and_validation(gpu_ctx):
    """G = 2 groups in one launch (CSR over (g, r, k) spanning them, the outer pool with offsets);
    a malformed id_off is reported (flags bit 5), an int32 one refused."""
    R, K, K2, A = 12, 3, 4, 4
    parts = [O.nested_map_objects(R, K, K2, A, seed=70 + g, steps=160) for g in range(2)]
    allm = parts[0] + parts[1]
    V = max([len(ie.val.vals) for m in allm for e in m.entries.values() for ie in e.val.entries.values()] + [1])
    d = O.nested_map_to_dense(allm, K, K2, A, V)
    off = [0, sum(len(m.deferred) for m in parts[0]), sum(len(m.deferred) for m in allm)]
    d["def_row"] = d["def_row"] % R
    shp = lambda x: to_dev(x.reshape((2, R) + x.shape[1:]))  # noqa: E731
    Dn = off[-1]
    kw = dict(def_off=off, def_row=torch.from_numpy(d["def_row"].astype(np.int32)).cuda(),
              def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"])) if Dn else {}
    Di = d["id_clock"].shape[0]
    ikw = dict(id_clock=to_dev(d["id_clock"]), id_keys=to_dev(d["id_keys"])) if Di else {}
    args = [shp(d[x]) for x in ("clock", "ec", "ic", "iec", "ivc", "ivv")]
    res = cg.map.nested_lub_many(*args, to_dev(d["id_off"]), ctx=gpu_ctx, **ikw, **kw)
    for g in range(2):
        dset = []
        if Dn:
            dset = [(np.array(rm, np.uint64), ks) for rm, ks in
                    cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys, off[g], off[g + 1])]
        idn = res.id_n.cpu().numpy()[g]
        idc, idk = to_host(res.id_clock)[g], to_host(res.id_keys)[g]
        idef = {k: [(idc[k, i], O.bitmap_members(idk[k, i:i + 1])) for i in range(int(idn[k]))] for k in range(K)}
        got = O.dense_to_nested_map(to_host(res.clock)[g], to_host(res.ec)[g], to_host(res.ic)[g],
                                    to_host(res.iec)[g], to_host(res.ivc)[g], to_host(res.ivv)[g],
                                    res.nval.cpu().numpy()[g], idef, dset)
        assert canon(got) == canon(O.map_fold_objects(parts[g]))
    off32 = torch.from_numpy(d["id_off"].astype(np.int32)).cuda()
    with pytest.raises(ValueError, match="int64"):
        cg.map.nested_lub_many(*args, off32, ctx=gpu_ctx, **ikw, **kw)
    if Di >= 1:
        bad = d["id_off"].copy()
        bad[-1] += np.uint64(1)  # last entry past the rows
        with pytest.raises(ValueError, match="id_off invalid"):
            cg.map.nested_lub_many(*args, to_dev(bad), ctx=gpu_ctx, **ikw, **kw)


def test_map_nested_empty(gpu_ctx):
    """R = 0 folds to Map::new()."""
    z = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    res = cg.map.nested_lub_many(z(2, 0, 4), z(2, 0, 3, 4), z(2, 0, 3, 4), z(2, 0, 3, 2, 4), z(2, 0, 3, 2, 1, 4),
                                 z(2, 0, 3, 2, 1), z(1), ctx=gpu_ctx)
    assert not to_host(res.clock).any() and not to_host(res.ec).any() and not to_host(res.iec).any()
    assert not res.nval.cpu().numpy().any() and not res.id_n.cpu().numpy().any()
