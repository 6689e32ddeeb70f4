"""Pins the MVReg / Map restatement in oracle/oracle.py to the reference's own tests.

Every test below restates one reference test (cited file:line) against the oracle types;
the quickcheck properties (test/map.rs:524-827, test/mvreg.rs:142-304) are replayed over
seeded random inputs drawn like quickcheck's (u8 tuples, vectors of up to ~40 ops).
Config 4 of BASELINE.json is Map<u32, MVReg<u64>>; these tests also cover the nested
Map<u8, Map<u8, MVReg<u8>>> the reference's tests use, since the restatement is generic.
"""
import random

import pytest

import oracle as O
from oracle import Dot, Map, MapRm, MapUp, MVReg, MVRegPut, RmCtx, VClock


def vc(*dots):
    return VClock.from_dots(Dot(a, c) for a, c in dots)


def TMap():  # test/map.rs:9  Map<u8, Map<u8, MVReg<u8, u8>>, u8>
    return Map(lambda: Map(MVReg))


def apply_ops(m, ops):  # test/map.rs:473-477
    for op in ops:
        m.apply(op)


def build_ops(actor, ops_data):
    """test/map.rs:11-46."""
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


def read_nested(m, k1, k2):
    v = m.get(k1).val
    if v is None:
        return None
    r = v.get(k2).val
    return None if r is None else r.read().val


# ---- src/map.rs in-module tests ----------------------------------------------------------
def test_get():  # map.rs:361-379
    m = TMap()
    assert m.get(0).val is None
    m.clock.apply(m.clock.inc(1))
    m.entries[0] = O.MapEntry(m.clock.copy(), Map(MVReg))
    assert m.get(0).val == Map(MVReg)


def test_op_exchange_converges_quickcheck1():  # map.rs:381-434
    op_actor1 = MapUp(Dot(0, 3), 9, MapUp(Dot(0, 3), 0, MVRegPut(vc((0, 3)), 0)))
    op_1_actor2 = MapUp(Dot(1, 1), 9, MapRm(vc((1, 1)), {0}))
    op_2_actor2 = MapRm(vc((1, 2)), {9})
    m1, m2 = TMap(), TMap()
    m1.apply(op_actor1)
    assert m1.clock == vc((0, 3))
    assert m1.entries[9].clock == vc((0, 3))
    assert len(m1.entries[9].val.deferred) == 0
    m2.apply(op_1_actor2)
    m2.apply(op_2_actor2)
    assert m2.clock == vc((1, 1))
    assert 9 not in m2.entries
    assert m2.deferred.get(vc((1, 2))) == {9}
    m1.apply(op_1_actor2)
    m1.apply(op_2_actor2)
    m2.apply(op_actor1)
    assert m1 == m2


def test_merge_error():  # map.rs:436-494 (Map<u8, Orswot<u8, u8>, u8>)
    def orswot(clock, entries):
        o = O.Orswot()
        o.clock = clock
        o.entries = entries
        return o

    m1 = Map(O.Orswot)
    m1.clock = vc((75, 1))
    m2 = Map(O.Orswot)
    m2.clock = vc((75, 1), (93, 1))
    m2.entries = {101: O.MapEntry(vc((75, 1), (93, 1)),
                                  orswot(vc((75, 1), (93, 1)), {1: vc((75, 1)), 2: vc((93, 1))}))}
    m1.merge(m2.copy())
    exp = Map(O.Orswot)
    exp.clock = vc((75, 1), (93, 1))
    exp.entries = {101: O.MapEntry(vc((93, 1)), orswot(vc((93, 1)), {2: vc((93, 1))}))}
    assert m1 == exp
    m2.merge(m1.copy())
    assert m1 == m2


# ---- test/map.rs -----------------------------------------------------------------------------
def test_new():  # test/map.rs:49-53
    m = Map(MVReg)
    assert m.len().val == 0
    assert m.is_empty().val


def test_is_empty():  # test/map.rs:56-68
    m = Map(lambda: Map(MVReg))
    r = m.is_empty()
    assert r.val
    m.apply(m.update("user_32", r.derive_add_ctx("A"),
                     lambda mp, ctx: mp.update("name", ctx, lambda reg, c: reg.write("bob", c))))
    assert not m.is_empty().val


def test_update():  # test/map.rs:71-125
    m = TMap()
    ctx = m.get(101).derive_add_ctx(1)
    op = m.update(101, ctx, lambda mp, ctx: mp.update(110, ctx, lambda reg, c: reg.write(2, c)))
    assert op == MapUp(Dot(1, 1), 101, MapUp(Dot(1, 1), 110, MVRegPut(vc((1, 1)), 2)))
    assert m == TMap()
    m.apply(op)
    assert read_nested(m, 101, 110) == [2]

    def f(mp, ctx):
        def g(reg, c):
            assert reg.read().val == [2]
            return reg.write(6, c)
        return mp.update(110, ctx, g)

    m.apply(m.update(101, m.get(101).derive_add_ctx(1), f))
    assert read_nested(m, 101, 110) == [6]


def test_remove():  # test/map.rs:127-146
    m = TMap()
    add_ctx = m.len().derive_add_ctx(1)
    inner = Map(MVReg)
    inner.apply(inner.update(110, add_ctx, lambda r, c: r.write(0, c)))
    m.apply(m.update(101, add_ctx, lambda mp, c: mp.update(110, c, lambda r, c2: r.write(0, c2))))
    assert m.get(101).val == inner
    assert m.len().val == 1
    m.apply(m.rm(101, m.get(101).derive_rm_ctx()))
    assert m.get(101).val is None
    assert m.len().val == 0


def test_reset_remove_semantics():  # test/map.rs:148-174
    m1 = TMap()
    m1.apply(m1.update(101, m1.get(101).derive_add_ctx(74),
                       lambda mp, c: mp.update(110, c, lambda r, c2: r.write(32, c2))))
    m2 = m1.copy()
    m1.apply(m1.rm(101, m1.get(101).derive_rm_ctx()))
    m2.apply(m2.update(101, m2.get(101).derive_add_ctx(37),
                       lambda mp, c: mp.update(220, c, lambda r, c2: r.write(5, c2))))
    snap = m1.copy()
    m1.merge(m2.copy())
    m2.merge(snap)
    assert m1 == m2
    inner = m1.get(101).val
    assert inner.get(220).val.read().val == [5]
    assert inner.get(110).val is None
    assert inner.len().val == 1


def test_updating_with_current_clock_should_be_a_nop():  # test/map.rs:176-195
    m1 = TMap()
    m1.apply(MapUp(Dot(1, 0), 0, MapUp(Dot(1, 0), 1, MVRegPut(VClock(), 235))))
    assert m1 == TMap()


def test_concurrent_update_and_remove_add_bias():  # test/map.rs:197-235
    m1, m2 = TMap(), TMap()
    op1 = MapRm(vc((1, 1)), {102})
    op2 = m2.update(102, m2.get(102).derive_add_ctx(2),
                    lambda mp, c: mp.update(42, c, lambda r, c2: r.write(7, c2)))
    m1.apply(op1)
    m2.apply(op2)
    m1c, m2c = m1.copy(), m2.copy()
    m1c.merge(m2.copy())
    m2c.merge(m1.copy())
    m1.apply(op2)
    m2.apply(op1)
    assert m1c == m2c
    assert m1 == m2
    assert m1 == m1c
    assert read_nested(m1, 102, 42) == [7]


def test_op_exchange_commutes_quickcheck1():  # test/map.rs:237-263
    m1 = Map(MVReg)
    m1_op1 = m1.update(0, m1.get(0).derive_add_ctx(1), lambda r, c: r.write(0, c))
    m1.apply(m1_op1)
    m1_op2 = m1.rm(0, m1.get(0).derive_rm_ctx())
    m1.apply(m1_op2)
    m2 = Map(MVReg)
    m2_op1 = m2.update(0, m2.get(0).derive_add_ctx(2), lambda r, c: r.write(0, c))
    m2.apply(m2_op1)
    m1.apply(m2_op1)
    m2.apply(m1_op1)
    m2.apply(m1_op2)
    assert m1 == m2


def test_op_deferred_remove():  # test/map.rs:265-300
    m1 = Map(MVReg)
    m2, m3 = m1.copy(), m1.copy()
    up1 = m1.update(0, m1.get(0).derive_add_ctx(1), lambda r, c: r.write(0, c))
    m1.apply(up1)
    up2 = m1.update(1, m1.get(1).derive_add_ctx(1), lambda r, c: r.write(1, c))
    m1.apply(up2)
    m2.apply(up1)
    m2.apply(up2)
    rm = m2.rm(0, m2.get(0).derive_rm_ctx())
    m2.apply(rm)
    assert m2.get(0).val is None
    m3.apply(rm)
    m3.apply(up1)
    m3.apply(up2)
    m1.apply(rm)
    assert m2.get(0).val is None
    assert m3.get(1).val.read().val == [1]
    assert m2 == m3
    assert m1 == m2
    assert m1 == m3


def test_merge_deferred_remove():  # test/map.rs:302-329
    m1, m2, m3 = Map(MVReg), Map(MVReg), Map(MVReg)
    m1.apply(m1.update(0, m1.get(0).derive_add_ctx(1), lambda r, c: r.write(0, c)))
    m1.apply(m1.update(1, m1.get(1).derive_add_ctx(1), lambda r, c: r.write(1, c)))
    m2.merge(m1.copy())
    m2.apply(m2.rm(0, m2.get(0).derive_rm_ctx()))
    assert m2.get(0).val is None
    m3.merge(m2.copy())
    m3.merge(m1.copy())
    m1.merge(m2.copy())
    assert m2.get(0).val is None
    assert m3.get(1).val.read().val == [1]
    assert m2 == m3
    assert m1 == m2
    assert m1 == m3


def test_commute_quickcheck_bug():  # test/map.rs:331-362
    ops = [MapRm(vc((45, 1)), {0}),
           MapUp(Dot(45, 2), 0, MapUp(Dot(45, 1), 0, MVRegPut(VClock(), 0)))]
    m = TMap()
    apply_ops(m, ops)
    snap = m.copy()
    empty = TMap()
    m.merge(empty.copy())
    empty.merge(snap)
    assert m == empty


def test_idempotent_quickcheck_bug1():  # test/map.rs:364-404
    ops = [MapUp(Dot(21, 5), 0, MapUp(Dot(21, 1), 32, MVRegPut(VClock(), 42))),
           MapRm(vc((21, 5)), {0}),
           MapUp(Dot(21, 6), 1, MapUp(Dot(21, 1), 0, MVRegPut(VClock(), 0)))]
    m = TMap()
    apply_ops(m, ops)
    snap = m.copy()
    m.merge(snap.copy())
    assert m == snap


def test_idempotent_quickcheck_bug2():  # test/map.rs:406-430
    m = TMap()
    m.apply(MapUp(Dot(32, 5), 0, MapUp(Dot(32, 5), 0, MVRegPut(VClock(), 0))))
    snap = m.copy()
    m.merge(snap.copy())
    assert m == snap


def test_op_exchange_same_as_merge_quickcheck1():  # test/map.rs:432-478
    op1 = MapUp(Dot(38, 4), 216, MapUp(Dot(38, 1), 37, MVRegPut(vc((38, 1)), 94)))
    op2 = MapUp(Dot(91, 9), 216, MapUp(Dot(91, 1), 37, MVRegPut(vc((91, 1)), 94)))
    m1, m2 = TMap(), TMap()
    m1.apply(op1)
    m2.apply(op2)
    m1m = m1.copy()
    m1m.merge(m2.copy())
    m2m = m2.copy()
    m2m.merge(m1.copy())
    m1.apply(op2)
    m2.apply(op1)
    assert m1 == m2
    assert m1m == m2m
    assert m1 == m1m and m2 == m2m and m1 == m2m and m2 == m1m


def test_idempotent_quickcheck1():  # test/map.rs:480-516
    ops = [MapUp(Dot(62, 9), 47, MapUp(Dot(62, 1), 65, MVRegPut(vc((62, 1)), 240))),
           MapUp(Dot(62, 11), 60, MapUp(Dot(62, 1), 193, MVRegPut(vc((62, 1)), 28)))]
    m = TMap()
    apply_ops(m, ops)
    snap = m.copy()
    m.merge(snap.copy())
    assert m == snap


# ---- quickcheck properties of test/map.rs, replayed over seeded inputs -------------------
def _prim(rng, n_max=40):
    actor = rng.randrange(256)
    ops = [tuple(rng.randrange(256) for _ in range(5)) for _ in range(rng.randrange(n_max))]
    # quickcheck's u8 generator favours small values; mix both regimes for keys
    if rng.random() < 0.5:
        ops = [(c, ic, k % 4, ik % 4, v) for c, ic, k, ik, v in ops]
    return actor, ops


def _maps(rng, n):
    while True:
        prims = [_prim(rng) for _ in range(n)]
        actors = [p[0] for p in prims]
        if len(set(actors)) == n:  # the props discard equal actors
            return [build_ops(*p)[1] for p in prims]


CASES = range(60)


@pytest.mark.parametrize("seed", CASES)
def test_prop_map_merge_laws(seed):
    """prop_op_exchange_same_as_merge, prop_merge_commutative, prop_merge_associative,
    prop_merge_followed_by_merge, prop_merge_idempotent, prop_op_idempotent
    (test/map.rs:526-550, :694-721, :660-692, :723-748, :750-764, :613-624)."""
    rng = random.Random(seed)
    ops1, ops2, ops3 = _maps(rng, 3)
    m1, m2, m3 = TMap(), TMap(), TMap()
    apply_ops(m1, ops1)
    apply_ops(m2, ops2)
    apply_ops(m3, ops3)
    # idempotent (merge and op)
    for m, ops in ((m1, ops1), (m2, ops2)):
        x = m.copy()
        x.merge(m.copy())
        assert x == m
        y = m.copy()
        apply_ops(y, ops)
        assert y == m
    # op exchange == merge
    mm = m1.copy()
    mm.merge(m2.copy())
    a, b = m1.copy(), m2.copy()
    apply_ops(a, ops2)
    apply_ops(b, ops1)
    assert a == mm and b == mm
    # commutative, followed-by-merge
    x, y = m1.copy(), m2.copy()
    x.merge(m2.copy())
    y.merge(m1.copy())
    assert x == y
    x, y = m1.copy(), m2.copy()
    x.merge(y.copy())
    y.merge(x.copy())
    assert x == y
    # associative
    l, r = m1.copy(), m2.copy()
    l.merge(m2.copy())
    l.merge(m3.copy())
    r.merge(m3.copy())
    r2 = m1.copy()
    r2.merge(r)
    assert l == r2


@pytest.mark.parametrize("seed", range(30))
def test_prop_map_forget(seed):
    """prop_forget_with_empty_vclock_is_nop, prop_forget_with_map_clock_is_empty_map,
    prop_forget_than_merge_same_as_merge_than_forget (test/map.rs:766-826)."""
    rng = random.Random(1000 + seed)
    ops1, ops2 = _maps(rng, 2)
    m1, m2 = TMap(), TMap()
    apply_ops(m1, ops1)
    apply_ops(m2, ops2)
    x = m1.copy()
    x.forget(VClock())
    assert x == m1
    x = m1.copy()
    x.forget(x.len().rm_clock)
    assert x.len().val == 0
    clock = VClock.from_dots(Dot(a, c) for a, c in zip(
        [rng.randrange(256) for _ in range(6)], [rng.randrange(256) for _ in range(6)]))
    fa1, fa2 = m1.copy(), m2.copy()
    m1.forget(clock)
    m2.forget(clock)
    m1.merge(m2)
    fa1.merge(fa2)
    fa1.forget(clock)
    assert fa1 == m1


# ---- test/mvreg.rs ---------------------------------------------------------------------------
def test_mvreg_doctest():  # mvreg.rs:13-31
    r1 = MVReg()
    r2 = r1.copy()
    c1, c2 = r1.read(), r2.read()
    r1.apply(r1.write("bob", c1.derive_add_ctx(123)))
    op = r2.write("alice", c2.derive_add_ctx(111))
    r2.apply(op)
    r1.apply(op)
    assert r1.read().val == ["bob", "alice"]


def test_mvreg_apply():  # test/mvreg.rs:12-22
    reg = MVReg()
    clock = vc((2, 1))
    reg.apply(MVRegPut(clock, 71))
    assert reg.read().add_clock == clock
    assert reg.read().val == [71]


def test_mvreg_write_should_not_mutate_reg():  # test/mvreg.rs:24-35
    reg = MVReg()
    op = reg.write(32, reg.read().derive_add_ctx("A"))
    assert reg == MVReg()
    reg.apply(op)
    assert reg.read().val == [32]
    assert reg.read().add_clock == vc(("A", 1))


@pytest.mark.parametrize("via", ["merge", "apply"])
def test_mvreg_concurrent_same_value_dont_collapse(via):  # test/mvreg.rs:37-72
    r1, r2 = MVReg(), MVReg()
    r1.apply(r1.write(23, r1.read().derive_add_ctx("A")))
    if via == "merge":
        r2.apply(r2.write(23, r2.read().derive_add_ctx("B")))
        r1.merge(r2)
    else:
        r1.apply(r2.write(23, r2.read().derive_add_ctx("B")))
    assert r1.read().val == [23, 23]
    assert r1.read().add_clock == vc(("A", 1), ("B", 1))


def test_mvreg_multi_val():  # test/mvreg.rs:74-84
    r1, r2 = MVReg(), MVReg()
    r1.apply(r1.write(32, r1.read().derive_add_ctx("A")))
    r2.apply(r2.write(82, r2.read().derive_add_ctx("B")))
    r1.merge(r2)
    assert r1.read().val in ([32, 82], [82, 32])


def test_mvreg_op_commute_quickcheck1():  # test/mvreg.rs:86-105
    reg1, reg2 = MVReg(), MVReg()
    op1 = MVRegPut(vc(("A", 1)), 1)
    op2 = MVRegPut(vc(("B", 1)), 2)
    reg2.apply(op2)
    reg2.apply(op1)
    reg1.apply(op1)
    reg1.apply(op2)
    assert reg1 == reg2


def _ops_not_compatible(opss):  # test/mvreg.rs:107-128
    for a_ops in opss:
        for b_ops in opss:
            if b_ops == a_ops:
                continue
            ac, bc = VClock(), VClock()
            for (_, aa), (_, ba) in zip(a_ops, b_ops):
                ac.apply(ac.inc(aa))
                bc.apply(bc.inc(ba))
                if bc.get(aa) == ac.get(aa):
                    return True
    return False


def _build_reg(prim):  # test/mvreg.rs:129-140
    reg, ops = MVReg(), []
    for val, actor in prim:
        op = reg.write(val, reg.read().derive_add_ctx(actor))
        reg.apply(op)
        ops.append(op)
    return reg, ops


@pytest.mark.parametrize("seed", range(60))
def test_prop_mvreg_laws(seed):
    """test/mvreg.rs:142-304: set_with_ctx_from_read, merge idempotent / commutative /
    associative, forget, op idempotent / commutative / associative."""
    rng = random.Random(5000 + seed)
    nact = rng.choice([3, 8, 256])

    def prim():
        return [(rng.randrange(256), rng.randrange(nact)) for _ in range(rng.randrange(12))]

    p1, p2, p3 = prim(), prim(), prim()
    reg, ops = _build_reg(p1)
    r = reg.copy()
    r.apply(r.write(23, r.read().derive_add_ctx(rng.randrange(256))))
    assert r.read().val == [23]
    x = reg.copy()
    x.merge(reg.copy())
    assert x == reg
    x = reg.copy()
    for op in ops:
        x.apply(op)
    assert x == reg
    x = reg.copy()
    x.forget(VClock())
    assert x == reg
    x.forget(x.read().add_clock)
    assert x == MVReg()
    if _ops_not_compatible([p1, p2, p3]):
        return
    (r1, o1), (r2, o2), (r3, o3) = _build_reg(p1), _build_reg(p2), _build_reg(p3)
    a, b = r1.copy(), r2.copy()
    a.merge(r2.copy())
    b.merge(r1.copy())
    assert a == b
    a = r1.copy()
    a.merge(r2.copy())
    a.merge(r3.copy())
    b = r2.copy()
    b.merge(r3.copy())
    b.merge(r1.copy())
    assert a == b
    a, b = r1.copy(), r2.copy()
    for op in o2:
        a.apply(op)
    for op in o1:
        b.apply(op)
    assert a == b
    for op in o3:
        a.apply(op)
    c = r2.copy()
    for op in o3:
        c.apply(op)
    for op in o1:
        c.apply(op)
    assert a == c
