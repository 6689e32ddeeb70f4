"""CPU: the oracle's bincode restatement (test infrastructure for the wire ingest / egress) —
hand-computed byte layouts of small states and decode(encode(x)) == x."""
import struct

import numpy as np

import oracle as O


def test_vclock_bytes_by_hand():
    # BTreeMap<u32, u64> {1: 5, 7: 2^40}: u64 len 2, then (1u32, 5u64), (7u32, 2^40 u64), ascending
    b = O.bc_vclock({7: 2**40, 1: 5})
    assert b == (b"\x02" + b"\x00" * 7 + b"\x01\x00\x00\x00" + b"\x05" + b"\x00" * 7
                 + b"\x07\x00\x00\x00" + struct.pack("<Q", 2**40))
    assert O.bc_vclock({}) == b"\x00" * 8
    assert O.bc_vclock({3: 0}) == b"\x00" * 8  # an absent actor (0) is not stored (vclock.rs:156)


def test_struct_layouts():
    assert O.bc_lwwreg(9, 2) == struct.pack("<QQ", 9, 2)                     # val, marker
    assert O.bc_pncounter({1: 1}, {2: 3}) == O.bc_vclock({1: 1}) + O.bc_vclock({2: 3})  # p then n
    assert O.bc_gset({5, 1}) == struct.pack("<QQQ", 2, 1, 5)
    b = O.bc_orswot({0: 2}, {10: {0: 2}}, [({1: 4}, [10, 11])])
    assert b == (O.bc_vclock({0: 2}) + struct.pack("<QQ", 1, 10) + O.bc_vclock({0: 2}) + struct.pack("<Q", 1)
                 + O.bc_vclock({1: 4}) + struct.pack("<QQQ", 2, 10, 11))


def test_round_trips():
    rng = np.random.default_rng(0)
    for _ in range(50):
        dots = {int(a): int(c) for a, c in zip(rng.integers(0, 2**32, 20), rng.integers(1, 2**63, 20))}
        assert O.unbc_vclock(O.bc_vclock(dots))[0] == dots
        s = set(int(x) for x in rng.integers(0, 2**63, 30))
        assert O.unbc_gset(O.bc_gset(s))[0] == s
        ent = {int(m): {int(a): int(rng.integers(1, 99))} for m, a in zip(rng.integers(0, 2**60, 5), range(5))}
        de = [({9: 3}, [1, 2]), ({9: 3}, [4]), ({8: 1}, [])]
        c, e, d, pos = O.unbc_orswot(O.bc_orswot({1: 1}, ent, de, order=list(ent)[::-1]))
        assert c == {1: 1} and e == ent and d == {((9, 3),): {1, 2, 4}, ((8, 1),): set()}


def test_map_bincode_round_trip_and_layout():
    """Map<u32, MVReg<u64>> (map.rs:31-47, mvreg.rs:32-35): the restated bincode form decodes to
    what was encoded, keys ascending (BTreeMap), values in Vec order, and its byte layout is the
    derive's field order (clock, entries, deferred)."""
    clock = {7: 3, 2: 9}
    entries = {40: ({2: 9}, [({2: 9}, 11), ({7: 3}, 12)]), 5: ({7: 1}, [])}
    deferred = [({2: 10}, [40, 5])]
    b = O.bc_map(clock, entries, deferred)
    c, e, d, pos = O.unbc_map(b)
    assert pos == len(b) and len(b) % 4 == 0
    assert c == clock and e == entries and d == {((2, 10),): {5, 40}}
    import struct
    # clock: 2 dots ascending by actor
    assert struct.unpack_from("<QIQIQ", b, 0) == (2, 2, 9, 7, 3)
    # entries: count, then key 5 first
    assert struct.unpack_from("<QI", b, 32) == (2, 5)


def test_value_map_bincode_round_trips_and_layout():
    """Map<u32, GCounter / PNCounter / Orswot<u64>> (map.rs:31-47 with gcounter.rs:25-28,
    pncounter.rs:28-32, orswot.rs:20-25 as the value): decode(encode(m)) == m over op-replay states
    with deferred removes at both levels, and the byte layout of a small one by hand."""
    aid = [3, 10, 11, 40, 41, 90]
    kid = [2, 7, 8, 100, 101]
    mid = [5, 6, 2**40, 2**40 + 1, 2**62]
    for W, vnew in ((1, O.GCounter), (2, O.PNCounter)):
        maps = O.map_counter_objects(12, 5, 6, W, seed=40, steps=200)
        assert sum(len(m.deferred) for m in maps) > 0
        for m in maps:
            b = O.bc_map_obj(m, aid, kid)
            got, pos = O.unbc_map_obj(b, vnew, aid, kid)
            assert pos == len(b) and got == m
    maps = O.map_orswot_objects(12, 5, 5, 6, seed=55, steps=200, p_vrm=0.45)
    assert sum(len(e.val.deferred) for m in maps for e in m.entries.values()) > 0
    for m in maps:
        b = O.bc_map_obj(m, aid, kid, mid)
        got, pos = O.unbc_map_obj(b, O.Orswot, aid, kid, mid)
        assert pos == len(b) and got == m
    # by hand: Map<u32, PNCounter>: clock {a0: 2}, key 1 -> (entry clock {a0: 2}, p {a0: 1}, n {a0: 1})
    m = O.Map(O.PNCounter)
    m.clock = O.VClock({0: 2})
    v = O.PNCounter()
    v.p.inner, v.n.inner = O.VClock({0: 1}), O.VClock({0: 1})
    m.entries[1] = O.MapEntry(O.VClock({0: 2}), v)
    m.deferred[O.VClock({1: 4})] = {0, 2}
    b = O.bc_map_obj(m, aid, kid)
    assert b == (O.bc_vclock({3: 2}) + struct.pack("<QI", 1, 7) + O.bc_vclock({3: 2}) + O.bc_vclock({3: 1})
                 + O.bc_vclock({3: 1}) + struct.pack("<Q", 1) + O.bc_vclock({10: 4}) + struct.pack("<QII", 2, 2, 8))


def test_nested_map_bincode_round_trip():
    """Map<u32, Map<u32, MVReg<u64>>> (the reference's TMap, test/map.rs:10): decode(encode(m)) == m
    over op-replay states with inner and outer deferred removes, registers in Vec order."""
    aid = [3, 10, 11, 40, 41, 90]
    kid = [2, 7, 8, 100, 101]
    iid = [1, 4, 9, 16, 25, 36, 49]
    maps = O.nested_map_objects(16, 5, 7, 6, seed=33, steps=220, p_irm=0.5, p_ooo=0.8, p_rm=0.3)
    assert sum(len(e.val.deferred) for m in maps for e in m.entries.values()) > 0
    for m in maps:
        b = O.bc_map_obj(m, aid, kid, iid=iid)
        got, pos = O.unbc_map_obj(b, "nested", aid, kid, iid=iid)
        assert pos == len(b) and got == m
        for k, e in m.entries.items():
            for j, ie in e.val.entries.items():
                assert [x for _, x in got.entries[k].val.entries[j].val.vals] == [x for _, x in ie.val.vals]
