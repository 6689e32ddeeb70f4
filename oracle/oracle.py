"""ORACLE — test infrastructure only (never imported by the product package).

Pure-Python restatement of the reference `crdts` 3.0.0 (rust-crdt) types on the merge path,
statement by statement, plus numpy restatements of the synthetic-input hash used by the GPU
generators and ctypes access to the C++ twin (oracle/ref_fold.cpp).

Pinned by the reference's own known-answer tests, transcribed in tests/golden/kat_*.json
(test/vclock.rs, test/orswot.rs, src/orswot.rs, src/gcounter.rs, src/pncounter.rs,
src/lwwreg.rs, src/gset.rs doctests) — see tests/test_oracle_kat.py.  The reference crate
itself cannot be built or run here (Rust; no cargo/rustc in the image).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Hashable, Iterable, Optional, Set, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# Ordering results of VClock.partial_cmp (vclock.rs:68-80)
LESS, EQUAL, GREATER, NONE = -1, 0, 1, None


class ConflictingMarker(Exception):
    """error.rs:8-15 Error::ConflictingMarker."""


# ---------------------------------------------------------------------------------------
# VClock  (src/vclock.rs)
# ---------------------------------------------------------------------------------------
class Dot:
    __slots__ = ("actor", "counter")

    def __init__(self, actor, counter: int):  # vclock.rs:40-45
        self.actor = actor
        self.counter = counter

    def __eq__(self, o):
        return isinstance(o, Dot) and (self.actor, self.counter) == (o.actor, o.counter)

    def __repr__(self):
        return f"Dot({self.actor!r}, {self.counter})"


class VClock:
    """vclock.rs:56-60: `dots: BTreeMap<A, u64>`; absent actor == 0."""

    __slots__ = ("dots",)

    def __init__(self, dots: Optional[Dict[Hashable, int]] = None):
        self.dots: Dict[Hashable, int] = dict(dots or {})

    @classmethod
    def from_dots(cls, dots: Iterable[Dot]) -> "VClock":  # FromIterator, vclock.rs:297-307
        v = cls()
        for d in dots:
            v.apply(d)
        return v

    def copy(self) -> "VClock":
        return VClock(self.dots)

    def __eq__(self, o):  # derived PartialEq on the BTreeMap
        return isinstance(o, VClock) and self.dots == o.dots

    def __hash__(self):  # derived Hash
        return hash(frozenset(self.dots.items()))

    def __repr__(self):
        return "VClock(%r)" % dict(sorted(self.dots.items(), key=lambda kv: repr(kv[0])))

    def get(self, actor) -> int:  # vclock.rs:207-209
        return self.dots.get(actor, 0)

    def is_empty(self) -> bool:  # vclock.rs:212-214
        return not self.dots

    def apply_dot(self, dot: Dot) -> None:  # vclock.rs:155-159
        if self.get(dot.actor) < dot.counter:
            self.dots[dot.actor] = dot.counter

    def apply(self, dot: Dot) -> None:  # CmRDT::apply vclock.rs:125-127
        self.apply_dot(dot)

    def merge(self, other: "VClock") -> None:  # CvRDT::merge vclock.rs:130-136
        for actor, counter in list(other.dots.items()):
            self.apply_dot(Dot(actor, counter))

    def inc(self, actor) -> Dot:  # vclock.rs:183-189
        return Dot(actor, self.get(actor) + 1)

    def forget(self, other: "VClock") -> None:  # Causal::forget vclock.rs:95-105
        for actor, counter in list(other.dots.items()):
            if counter >= self.get(actor):
                self.dots.pop(actor, None)

    def clone_without(self, base: "VClock") -> "VClock":  # vclock.rs:148-152
        c = self.copy()
        c.forget(base)
        return c

    @staticmethod
    def intersection(left: "VClock", right: "VClock") -> "VClock":  # vclock.rs:218-227
        return VClock({a: c for a, c in left.dots.items() if right.get(a) == c})

    def glb(self, other: "VClock") -> None:  # vclock.rs:246-259
        self.dots = {a: min(c, other.get(a)) for a, c in self.dots.items() if min(c, other.get(a)) != 0}

    def partial_cmp(self, other: "VClock"):  # vclock.rs:68-80
        if self == other:
            return EQUAL
        if all(self.get(w) >= c for w, c in other.dots.items()):
            return GREATER
        if all(other.get(w) >= c for w, c in self.dots.items()):
            return LESS
        return NONE

    def __ge__(self, other):
        return self.partial_cmp(other) in (GREATER, EQUAL)

    def __gt__(self, other):
        return self.partial_cmp(other) == GREATER

    def __le__(self, other):
        return self.partial_cmp(other) in (LESS, EQUAL)

    def __lt__(self, other):
        return self.partial_cmp(other) == LESS

    def concurrent(self, other) -> bool:  # vclock.rs:201-203
        return self.partial_cmp(other) is NONE


# ---------------------------------------------------------------------------------------
# GCounter / PNCounter / GSet / LWWReg
# ---------------------------------------------------------------------------------------
class GCounter:  # gcounter.rs:25-73
    def __init__(self):
        self.inner = VClock()

    def inc(self, actor) -> Dot:
        return self.inner.inc(actor)

    def apply(self, op: Dot) -> None:
        self.inner.apply(op)

    def merge(self, other: "GCounter") -> None:  # gcounter.rs:44-48
        self.inner.merge(other.inner)

    def read(self) -> int:  # gcounter.rs:70-72 (BigUint sum)
        return sum(self.inner.dots.values())

    def forget(self, clock: "VClock") -> None:  # Causal::forget gcounter.rs:50-54
        self.inner.forget(clock)

    def copy(self) -> "GCounter":
        g = GCounter()
        g.inner = self.inner.copy()
        return g

    def __eq__(self, o):
        return isinstance(o, GCounter) and self.inner == o.inner

    def __repr__(self):
        return f"GCounter({self.inner})"


class PNCounter:  # pncounter.rs:28-115
    POS, NEG = "Pos", "Neg"

    def __init__(self):
        self.p = GCounter()
        self.n = GCounter()

    def inc(self, actor):
        return (self.p.inc(actor), self.POS)

    def dec(self, actor):
        return (self.n.inc(actor), self.NEG)

    def apply(self, op) -> None:  # pncounter.rs:59-68
        dot, d = op
        (self.p if d == self.POS else self.n).apply(dot)

    def merge(self, other: "PNCounter") -> None:  # pncounter.rs:70-75
        self.p.merge(other.p)
        self.n.merge(other.n)

    def read(self) -> int:  # pncounter.rs:110-115
        return self.p.read() - self.n.read()

    def forget(self, clock: "VClock") -> None:  # Causal::forget pncounter.rs:77-82
        self.p.forget(clock)
        self.n.forget(clock)

    def copy(self) -> "PNCounter":
        c = PNCounter()
        c.p, c.n = self.p.copy(), self.n.copy()
        return c

    def __eq__(self, o):
        return isinstance(o, PNCounter) and self.p == o.p and self.n == o.n

    def __repr__(self):
        return f"PNCounter(p={self.p.inner}, n={self.n.inner})"


class GSet:  # gset.rs
    def __init__(self, items=()):
        self.value: Set = set(items)

    def insert(self, e) -> None:  # gset.rs:69-71
        self.value.add(e)

    def apply(self, op) -> None:
        self.insert(op)

    def merge(self, other: "GSet") -> None:  # gset.rs:38-40
        for e in other.value:
            self.insert(e)

    def contains(self, e) -> bool:
        return e in self.value


class LWWReg:  # lwwreg.rs
    def __init__(self, val, marker):
        self.val = val
        self.marker = marker

    def __eq__(self, o):
        return isinstance(o, LWWReg) and (self.val, self.marker) == (o.val, o.marker)

    def __repr__(self):
        return f"LWWReg(val={self.val!r}, marker={self.marker!r})"

    def update(self, val, marker) -> None:  # lwwreg.rs:84-98
        if self.marker < marker:
            self.val = val
            self.marker = marker
        elif self.marker == marker and val != self.val:
            raise ConflictingMarker()

    def merge(self, other: "LWWReg") -> None:  # lwwreg.rs:43-45
        self.update(other.val, other.marker)


# ---------------------------------------------------------------------------------------
# ctx.rs + Orswot (src/orswot.rs)
# ---------------------------------------------------------------------------------------
class ReadCtx:  # ctx.rs:12-21
    def __init__(self, add_clock: VClock, rm_clock: VClock, val):
        self.add_clock, self.rm_clock, self.val = add_clock, rm_clock, val

    def derive_add_ctx(self, actor) -> "AddCtx":  # ctx.rs:42-48
        clock = self.add_clock.copy()
        dot = clock.inc(actor)
        clock.apply(dot)
        return AddCtx(clock, dot)

    def derive_rm_ctx(self) -> "RmCtx":  # ctx.rs:50-54
        return RmCtx(self.rm_clock.copy())


class AddCtx:
    def __init__(self, clock: VClock, dot: Dot):
        self.clock, self.dot = clock, dot


class RmCtx:
    def __init__(self, clock: VClock):
        self.clock = clock


class OrswotAdd:  # orswot.rs:33-39
    def __init__(self, dot: Dot, members):
        self.dot, self.members = dot, set(members)


class OrswotRm:  # orswot.rs:40-46
    def __init__(self, clock: VClock, members):
        self.clock, self.members = clock, set(members)


class Orswot:
    """orswot.rs:20-25: clock, entries: HashMap<M, VClock>, deferred: HashMap<VClock, HashSet<M>>."""

    def __init__(self):
        self.clock = VClock()
        self.entries: Dict[Hashable, VClock] = {}
        self.deferred: Dict[VClock, Set] = {}

    def copy(self) -> "Orswot":
        o = Orswot()
        o.clock = self.clock.copy()
        o.entries = {m: c.copy() for m, c in self.entries.items()}
        o.deferred = {k.copy(): set(v) for k, v in self.deferred.items()}
        return o

    def __eq__(self, o):
        return (isinstance(o, Orswot) and self.clock == o.clock and self.entries == o.entries
                and self.deferred == o.deferred)

    def __repr__(self):
        return f"Orswot(clock={self.clock}, entries={self.entries}, deferred={self.deferred})"

    # CmRDT::apply  orswot.rs:55-79
    def apply(self, op) -> None:
        if isinstance(op, OrswotAdd):
            if self.clock.get(op.dot.actor) >= op.dot.counter:
                return
            for m in op.members:
                self.entries.setdefault(m, VClock()).apply(Dot(op.dot.actor, op.dot.counter))
            self.clock.apply(Dot(op.dot.actor, op.dot.counter))
            self.apply_deferred()
        else:
            self.apply_rm(set(op.members), op.clock.copy())

    # CvRDT::merge  orswot.rs:81-149
    def merge(self, other: "Orswot") -> None:
        other = other.copy()  # merge consumes `other` by value
        kept = {}
        for entry, clock in self.entries.items():  # :84-106
            if entry not in other.entries:
                if other.clock >= clock:
                    continue
                clock.forget(other.clock)
                kept[entry] = clock
            else:
                kept[entry] = clock
        self.entries = kept
        for entry, clock in other.entries.items():  # :108-138
            our = self.entries.get(entry)
            if our is not None:
                common = VClock.intersection(clock, our)
                common.merge(clock.clone_without(self.clock))
                common.merge(our.clone_without(other.clock))
                if common.is_empty():
                    del self.entries[entry]
                else:
                    self.entries[entry] = common
            else:
                if self.clock >= clock:
                    pass
                else:
                    clock.forget(self.clock)
                    self.entries[entry] = clock
        for rm_clock, members in other.deferred.items():  # :141-143
            self.apply_rm(set(members), rm_clock.copy())
        self.clock.merge(other.clock)  # :145
        self.apply_deferred()  # :147

    # orswot.rs:230-250
    def apply_rm(self, members: Set, clock: VClock) -> None:
        for m in members:
            mc = self.entries.get(m)
            if mc is not None:
                mc.forget(clock)
                if mc.is_empty():
                    del self.entries[m]
        if clock.partial_cmp(self.clock) in (NONE, GREATER):
            if clock in self.deferred:
                self.deferred[clock] |= members
            else:
                self.deferred[clock] = set(members)

    def apply_deferred(self) -> None:  # orswot.rs:281-286
        deferred, self.deferred = self.deferred, {}
        for clock, members in deferred.items():
            self.apply_rm(members, clock)

    def add(self, member, ctx: AddCtx) -> OrswotAdd:  # orswot.rs:196-201
        return OrswotAdd(ctx.dot, [member])

    def rm(self, member, ctx: RmCtx) -> OrswotRm:  # orswot.rs:212-219
        return OrswotRm(ctx.clock, [member])

    def contains(self, member) -> ReadCtx:  # orswot.rs:253-261
        mc = self.entries.get(member)
        return ReadCtx(self.clock.copy(), mc.copy() if mc is not None else VClock(), mc is not None)

    def read(self) -> ReadCtx:  # orswot.rs:264-270
        return ReadCtx(self.clock.copy(), self.clock.copy(), set(self.entries.keys()))

    def forget(self, clock: VClock) -> None:  # Causal::forget orswot.rs:150-183
        self.clock.forget(clock)
        kept = {}
        for m, mc in self.entries.items():
            mc = mc.copy()
            mc.forget(clock)
            if not mc.is_empty():
                kept[m] = mc
        self.entries = kept
        deferred = {}
        for rm, ms in self.deferred.items():
            rm = rm.copy()
            rm.forget(clock)
            if not rm.is_empty():
                deferred[rm] = ms
        self.deferred = deferred


# ---------------------------------------------------------------------------------------
# MVReg (src/mvreg.rs) and Map (src/map.rs) — config 4's Map<K, MVReg<V>>
# ---------------------------------------------------------------------------------------
class MVRegPut:  # mvreg.rs:38-47 Op::Put
    def __init__(self, clock: VClock, val):
        self.clock, self.val = clock, val

    def __eq__(self, o):
        return isinstance(o, MVRegPut) and (self.clock, self.val) == (o.clock, o.val)


class MVReg:
    """mvreg.rs:33-36: `vals: Vec<(VClock<A>, V)>` (ordered; equality is set-based)."""

    def __init__(self, vals=None):
        self.vals = [(c.copy(), v) for c, v in (vals or [])]

    def copy(self) -> "MVReg":
        return MVReg(self.vals)

    def __eq__(self, other):  # mvreg.rs:62-86 (order-free, each val unique)
        if not isinstance(other, MVReg):
            return False
        for a, b in ((self, other), (other, self)):
            for dot in a.vals:
                n = sum(1 for d in b.vals if d[0] == dot[0] and d[1] == dot[1])
                if n == 0:
                    return False
                assert n == 1, "MVReg sanity check (mvreg.rs:72)"
        return True

    def __repr__(self):
        return f"MVReg({self.vals})"

    def forget(self, clock: VClock) -> None:  # Causal::forget mvreg.rs:88-104
        out = []
        for vc, v in self.vals:
            vc = vc.copy()
            vc.forget(clock)
            if not vc.is_empty():
                out.append((vc, v))
        self.vals = out

    def merge(self, other: "MVReg") -> None:  # CvRDT::merge mvreg.rs:112-128
        other = other.copy()
        self.vals = [(c, v) for c, v in self.vals
                     if sum(1 for c2, _ in other.vals if c < c2) == 0]
        add = [(c, v) for c, v in other.vals
               if sum(1 for c1, _ in self.vals if c < c1) == 0
               and all(c != c1 for c1, _ in self.vals)]
        self.vals.extend(add)

    def apply(self, op: MVRegPut) -> None:  # CmRDT::apply mvreg.rs:130-166
        clock, val = op.clock.copy(), op.val
        if clock.is_empty():
            return
        self.vals = [(vc, v) for vc, v in self.vals if vc.partial_cmp(clock) in (NONE, GREATER)]
        should_add = True
        for vc, _ in self.vals:
            if vc > clock:
                should_add = False
        if should_add:
            self.vals.append((clock, val))

    def write(self, val, ctx: "AddCtx") -> MVRegPut:  # mvreg.rs:176-181
        return MVRegPut(ctx.clock.copy(), val)

    def clock(self) -> VClock:  # mvreg.rs:206-214
        acc = VClock()
        for c, _ in self.vals:
            acc.merge(c)
        return acc

    def read(self) -> ReadCtx:  # mvreg.rs:184-195
        c = self.clock()
        return ReadCtx(c, c.copy(), [v for _, v in self.vals])

    def read_ctx(self) -> ReadCtx:  # mvreg.rs:198-204
        c = self.clock()
        return ReadCtx(c, c.copy(), None)


class MapUp:  # map.rs:58-66 Op::Up
    def __init__(self, dot: Dot, key, op):
        self.dot, self.key, self.op = dot, key, op

    def __eq__(self, o):
        return isinstance(o, MapUp) and (self.dot, self.key, self.op) == (o.dot, o.key, o.op)


class MapRm:  # map.rs:51-57 Op::Rm
    def __init__(self, clock: VClock, keyset):
        self.clock, self.keyset = clock, set(keyset)

    def __eq__(self, o):
        return isinstance(o, MapRm) and (self.clock, self.keyset) == (o.clock, o.keyset)


class MapEntry:  # map.rs:40-47
    def __init__(self, clock: VClock, val):
        self.clock, self.val = clock, val

    def copy(self) -> "MapEntry":
        return MapEntry(self.clock.copy(), _deep(self.val))

    def __eq__(self, o):
        return isinstance(o, MapEntry) and self.clock == o.clock and self.val == o.val

    def __repr__(self):
        return f"Entry({self.clock}, {self.val})"


def _deep(x):
    return x.copy() if hasattr(x, "copy") else x


class Map:
    """map.rs:33-38: clock, entries: BTreeMap<K, Entry<V>>, deferred: HashMap<VClock, BTreeSet<K>>.

    `vnew` builds `V::default()` for the nested CRDT (MVReg, Map, Orswot, ...)."""

    def __init__(self, vnew=MVReg):
        self.vnew = vnew
        self.clock = VClock()
        self.entries: Dict[Hashable, MapEntry] = {}
        self.deferred: Dict[VClock, Set] = {}

    def copy(self) -> "Map":
        m = Map(self.vnew)
        m.clock = self.clock.copy()
        m.entries = {k: e.copy() for k, e in self.entries.items()}
        m.deferred = {c.copy(): set(ks) for c, ks in self.deferred.items()}
        return m

    def __eq__(self, o):  # derived PartialEq (map.rs:32)
        return (isinstance(o, Map) and self.clock == o.clock and self.entries == o.entries
                and self.deferred == o.deferred)

    def __repr__(self):
        return f"Map(clock={self.clock}, entries={self.entries}, deferred={self.deferred})"

    def forget(self, clock: VClock) -> None:  # Causal::forget map.rs:85-114
        kept = {}
        for k, e in self.entries.items():
            e = e.copy()
            e.clock.forget(clock)
            e.val.forget(clock)
            if not e.clock.is_empty():
                kept[k] = e
        self.entries = kept
        deferred = {}
        for rm, ks in self.deferred.items():
            rm = rm.copy()
            rm.forget(clock)
            if not rm.is_empty():
                deferred[rm] = ks
        self.deferred = deferred
        self.clock.forget(clock)

    def apply(self, op) -> None:  # CmRDT::apply map.rs:119-137
        if isinstance(op, MapRm):
            self.apply_keyset_rm(set(op.keyset), op.clock.copy())
            return
        dot = op.dot
        if self.clock.get(dot.actor) >= dot.counter:
            return
        e = self.entries.get(op.key)
        if e is None:
            e = self.entries[op.key] = MapEntry(VClock(), self.vnew())
        e.clock.apply(Dot(dot.actor, dot.counter))
        e.val.apply(op.op)
        self.clock.apply(Dot(dot.actor, dot.counter))
        self.apply_deferred()

    def merge(self, other: "Map") -> None:  # CvRDT::merge map.rs:140-220
        other = other.copy()
        kept = {}
        for key, entry in self.entries.items():  # :142-165
            if key not in other.entries:
                if other.clock >= entry.clock:
                    continue
                entry.clock.forget(other.clock)
                removed_information = other.clock.copy()
                removed_information.forget(entry.clock)
                entry.val.forget(removed_information)
                kept[key] = entry
            else:
                kept[key] = entry
        self.entries = kept
        for key, entry in other.entries.items():  # :167-210
            our = self.entries.get(key)
            if our is not None:
                common = VClock.intersection(entry.clock, our.clock)
                common.merge(entry.clock.clone_without(self.clock))
                common.merge(our.clock.clone_without(other.clock))
                if common.is_empty():
                    del self.entries[key]
                else:
                    our.val.merge(entry.val)
                    deleted = entry.clock.copy()
                    deleted.merge(our.clock.copy())
                    deleted.forget(common)
                    our.val.forget(deleted)
                    our.clock = common
            else:
                if self.clock >= entry.clock:
                    pass
                else:
                    entry.clock.forget(self.clock)
                    we_deleted = self.clock.copy()
                    we_deleted.forget(entry.clock)
                    entry.val.forget(we_deleted)
                    self.entries[key] = entry
        for rm_clock, keys in other.deferred.items():  # :213-215
            self.apply_keyset_rm(set(keys), rm_clock.copy())
        self.clock.merge(other.clock)  # :217
        self.apply_deferred()  # :219

    def is_empty(self) -> ReadCtx:  # map.rs:232-238
        return ReadCtx(self.clock.copy(), self.clock.copy(), not self.entries)

    def len(self) -> ReadCtx:  # map.rs:241-247
        return ReadCtx(self.clock.copy(), self.clock.copy(), len(self.entries))

    def get(self, key) -> ReadCtx:  # map.rs:250-260
        e = self.entries.get(key)
        return ReadCtx(self.clock.copy(), e.clock.copy() if e is not None else VClock(),
                       _deep(e.val) if e is not None else None)

    def update(self, key, ctx: "AddCtx", f) -> MapUp:  # map.rs:272-285
        e = self.entries.get(key)
        data = e.val if e is not None else self.vnew()
        return MapUp(Dot(ctx.dot.actor, ctx.dot.counter), key, f(data, ctx))

    def rm(self, key, ctx: "RmCtx") -> MapRm:  # map.rs:292-299
        return MapRm(ctx.clock.copy(), {key})

    def read_ctx(self) -> ReadCtx:  # map.rs:302-308
        return ReadCtx(self.clock.copy(), self.clock.copy(), None)

    def apply_deferred(self) -> None:  # map.rs:311-316
        deferred, self.deferred = self.deferred, {}
        for clock, keys in deferred.items():
            self.apply_keyset_rm(keys, clock)

    def apply_keyset_rm(self, keyset: Set, clock: VClock) -> None:  # map.rs:318-348
        for key in sorted(keyset, key=repr):
            e = self.entries.get(key)
            if e is not None:
                e.clock.forget(clock)
                if e.clock.is_empty():
                    del self.entries[key]
                else:
                    e.val.forget(clock)
        if self.clock.partial_cmp(clock) in (NONE, LESS):
            self.deferred.setdefault(clock, set()).update(keyset)


# ---------------------------------------------------------------------------------------
# Synthetic inputs: numpy restatement of rust-crdt_amd/csrc/synth.hip
# ---------------------------------------------------------------------------------------
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def mix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def synth_values(seed: int, idx: np.ndarray, kind: int) -> np.ndarray:
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = mix64(np.uint64(seed) + (idx + np.uint64(1)) * _GOLD)
    if kind == 0:
        v = h >> np.uint64(16)
        v = np.where(((h >> np.uint64(2)) & np.uint64(63)) == 0, h, v)
        return np.where((h & np.uint64(3)) == 0, np.uint64(0), v).astype(np.uint64)
    if kind == 1:
        return h & mix64(h ^ np.uint64(0x5851F42D4C957F2D))
    if kind == 2:
        return np.where((h >> np.uint64(58)) == 0, np.uint64(0xFFFFFFFFFFFF), h >> np.uint64(20)).astype(np.uint64)
    return np.where((h & np.uint64(1)) == 1, np.uint64(42), mix64(h ^ np.uint64(0x14057B7EF767814F))).astype(np.uint64)


def synth_matrix(seed: int, rows: int, width: int, kind: int, row0: int = 0) -> np.ndarray:
    """Rows [row0, row0+rows) of the (.. x width) synthetic matrix crdt_synth_fill writes."""
    idx = np.arange(row0 * width, (row0 + rows) * width, dtype=np.uint64)
    return synth_values(seed, idx, kind).reshape(rows, width)


def synth_orswot(seed: int, R: int, M: int, A: int, kmax: int, row0: int = 0):
    """Restatement of crdt_synth_orswot for replicas [row0, row0+R): (clock (R,A), entries (R,M,A))."""
    r = np.arange(row0, row0 + R, dtype=np.uint64)
    a = np.arange(A, dtype=np.uint64)
    m = np.arange(M, dtype=np.uint64)
    with np.errstate(over="ignore"):
        c = mix64(np.uint64(seed) + (r[:, None] * np.uint64(A) + a[None, :] + np.uint64(1)) * _GOLD)
    c = c % np.uint64(kmax + 1)
    pm = np.uint64(0x9E3779B1 % M)
    k = (m[:, None] + np.uint64(M) - (a[None, :] * pm) % np.uint64(M)) % np.uint64(M)  # (M, A)
    e = np.where((k[None] >= 1) & (k[None] <= c[:, None, :]), k[None], np.uint64(0))
    with np.errstate(over="ignore"):  # dot (m, a) removed w.p. 1/4, observed past k + 1 + delta
        hd = mix64(np.uint64(0xD1B54A32D192ED03) + m[:, None] * np.uint64(A) + a[None, :])  # (M, A)
    thr = k + np.uint64(1) + ((hd >> np.uint64(8)) & np.uint64(7))
    obs = ((hd & np.uint64(3)) == 0)[None] & (c[:, None, :] >= thr[None])
    e = np.where(obs, np.uint64(0), e).astype(np.uint64)
    return c.astype(np.uint64), e


def apply_rm_rows(entries: np.ndarray, rows, def_clock, def_members) -> np.ndarray:
    """forget(rm) of each deferred on its own replica's listed members (apply_rm's entry part)."""
    e = entries.copy()
    for d, r in enumerate(rows):
        for mm in bitmap_members(def_members[d]):
            row = e[r, mm]
            row[row <= def_clock[d]] = 0
    return e


# ---------------------------------------------------------------------------------------
# ctypes access to the C++ twin
# ---------------------------------------------------------------------------------------
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        # ORACLE_LIB: another build of the same source (tests/test_sanitizers.py loads the
        # -fsanitize=address,undefined one)
        path = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        S = ctypes.c_size_t
        L.oracle_vclock_fold.argtypes = [P, S, S, S, P]
        L.oracle_vclock_fold.restype = ctypes.c_double
        L.oracle_pncounter_fold.argtypes = [P, S, S, S, P]
        L.oracle_pncounter_fold.restype = ctypes.c_double
        L.oracle_gset_fold.argtypes = [P, S, S, S, P]
        L.oracle_gset_fold.restype = ctypes.c_double
        L.oracle_lwwreg_fold.argtypes = [P, P, S, P, P, P]
        L.oracle_lwwreg_fold.restype = ctypes.c_double
        L.oracle_vclock_merge_pairs.argtypes = [P, P, S, S]
        L.oracle_vclock_forget.argtypes = [P, P, S]
        L.oracle_vclock_partial_cmp.argtypes = [P, P, S]
        L.oracle_vclock_partial_cmp.restype = ctypes.c_int
        L.oracle_orswot_fold.argtypes = [P, P, S, S, S, P, P, P, P, P, P, P, S, ctypes.POINTER(S)]
        L.oracle_orswot_fold.restype = ctypes.c_double
        L.oracle_map_fold.argtypes = [P, P, P, P, S, S, S, S, P, P, P, S, P, P, P, P, P, P, P, S,
                                      ctypes.POINTER(S), P]
        L.oracle_map_fold.restype = ctypes.c_double
        L.oracle_orswot_apply_streams.argtypes = [S, S, S, P, P, P, P, P, P, P, P, P, P, P]
        L.oracle_orswot_apply_streams.restype = ctypes.c_double
        L.oracle_counter_fold_mt.argtypes = [P, S, S, S, ctypes.c_int, ctypes.c_int, P]
        L.oracle_counter_fold_mt.restype = ctypes.c_double
        L.oracle_dense_max_mt.argtypes = [P, S, S, S, ctypes.c_int, P]
        L.oracle_dense_max_mt.restype = ctypes.c_double
        I = ctypes.c_int
        L.oracle_orswot_fold_mt.argtypes = [P, P, S, S, S, P, P, P, I, P, P, P, P, S, ctypes.POINTER(S)]
        L.oracle_orswot_fold_mt.restype = ctypes.c_double
        L.oracle_map_fold_mt.argtypes = [P, P, P, P, S, S, S, S, P, P, P, S, I, P, P, P, P, P, P, P, S,
                                         ctypes.POINTER(S)]
        L.oracle_map_fold_mt.restype = ctypes.c_double
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64)


def vclock_fold(rows: np.ndarray) -> Tuple[np.ndarray, float]:
    """Left fold of VClock::merge from new() over the rows of a (R, A) u64 matrix."""
    rows = _c64(rows)
    R, A = rows.shape
    out = np.zeros(A, dtype=np.uint64)
    t = lib().oracle_vclock_fold(_p(rows), R, A, A, _p(out))
    return out, t


def counter_fold_mt(rows: np.ndarray, pn: bool, threads: int) -> Tuple[np.ndarray, float]:
    """The restated GCounter (pn=False) / PNCounter (pn=True, rows P | N) left fold split over
    `threads` host threads, partials merged at the end (oracle_counter_fold_mt)."""
    rows = _c64(rows)
    out = np.zeros(rows.shape[1], np.uint64)
    t = lib().oracle_counter_fold_mt(_p(rows), rows.shape[0], rows.shape[1], rows.shape[1], int(pn), int(threads),
                                     _p(out))
    return out, t


def dense_max_mt(rows: np.ndarray, threads: int) -> Tuple[np.ndarray, float]:
    """Elementwise max of dense u64 rows over `threads` host threads (oracle_dense_max_mt): the
    dense-SoA CPU fold of SURVEY §8d CPU timing (3).  Returns (max row, seconds)."""
    rows = _c64(rows)
    out = np.zeros(rows.shape[1], np.uint64)
    t = lib().oracle_dense_max_mt(_p(rows), rows.shape[0], rows.shape[1], rows.shape[1], int(threads), _p(out))
    return out, t


def pncounter_fold(rows: np.ndarray) -> Tuple[np.ndarray, float]:
    rows = _c64(rows)
    R, W = rows.shape
    out = np.zeros(W, dtype=np.uint64)
    t = lib().oracle_pncounter_fold(_p(rows), R, W // 2, W, _p(out))
    return out, t


def gset_fold(rows: np.ndarray) -> Tuple[np.ndarray, float]:
    rows = _c64(rows)
    R, W = rows.shape
    out = np.zeros(W, dtype=np.uint64)
    t = lib().oracle_gset_fold(_p(rows), R, W, W, _p(out))
    return out, t


def lwwreg_fold(marker: np.ndarray, val: np.ndarray) -> Tuple[int, int, int, float]:
    marker, val = _c64(marker), _c64(val)
    om, ov, fc = (np.zeros(1, dtype=np.uint64) for _ in range(3))
    t = lib().oracle_lwwreg_fold(_p(marker), _p(val), marker.size, _p(om), _p(ov), _p(fc))
    return int(om[0]), int(ov[0]), int(fc[0]), t


def vclock_merge_pairs(self_rows: np.ndarray, other_rows: np.ndarray) -> np.ndarray:
    s = _c64(self_rows).copy()
    o = _c64(other_rows)
    lib().oracle_vclock_merge_pairs(_p(s), _p(o), s.shape[0], s.shape[1])
    return s


def orswot_fold(clock: np.ndarray, entries: np.ndarray, def_off=None, def_clock=None,
                def_members=None, threads: Optional[int] = None):
    """Fold of Orswot::merge from new() over dense replicas.

    clock (R, A), entries (R, M, A); deferred pooled per replica as CSR def_off (R+1,),
    def_clock (D, A), def_members (D, Mw).  Returns (clock (A,), entries (M, A),
    deferred: set of (tuple rm clock, frozenset members), seconds).  `threads`: the multi-core
    baseline (ref_fold.cpp oracle_orswot_fold_mt: replica ranges folded per thread, the partial
    states then merged in order; same result).
    """
    clock, entries = _c64(clock), _c64(entries)
    R, M, A = entries.shape
    Mw = (M + 63) // 64
    if def_off is None:
        def_off = np.zeros(R + 1, dtype=np.uint64)
        def_clock = np.zeros((1, A), dtype=np.uint64)
        def_members = np.zeros((1, Mw), dtype=np.uint64)
    def_off, def_clock, def_members = _c64(def_off), _c64(def_clock), _c64(def_members)
    if def_off.shape != (R + 1,):  # per-replica offsets; anything else would be read out of bounds
        raise ValueError(f"orswot_fold: def_off must hold R + 1 = {R + 1} per-replica offsets, got {def_off.shape}")
    D = int(def_off[-1])
    maxd = max(D, 1)
    oc = np.zeros(A, dtype=np.uint64)
    oe = np.zeros((M, A), dtype=np.uint64)
    odc = np.zeros((maxd, A), dtype=np.uint64)
    odm = np.zeros((maxd, Mw), dtype=np.uint64)
    nd = ctypes.c_size_t(0)
    if threads is None:
        t = lib().oracle_orswot_fold(_p(clock), _p(entries), R, M, A, _p(def_off), _p(def_clock),
                                     _p(def_members), _p(oc), _p(oe), _p(odc), _p(odm), maxd,
                                     ctypes.byref(nd))
    else:
        t = lib().oracle_orswot_fold_mt(_p(clock), _p(entries), R, M, A, _p(def_off), _p(def_clock),
                                        _p(def_members), int(threads), _p(oc), _p(oe), _p(odc), _p(odm), maxd,
                                        ctypes.byref(nd))
    n = nd.value
    assert n <= maxd
    deferred = set()
    for k in range(n):
        deferred.add((tuple(int(x) for x in odc[k]), bitmap_members(odm[k])))
    return oc, oe, deferred, t


def orswot_apply_streams(N: int, M: int, A: int, op_off, kind, actor, counter, rm_row, rm_clock, mem_off, mem):
    """C++ twin: every state applies its op stream from Orswot::new() (orswot.rs:55-79) over
    std containers.  Arrays in the crdt_orswot_ops layout (numpy).  Returns
    (clock (N, A), entries (N, M, A), ndef (N,), apply seconds)."""
    out_c = np.zeros((N, A), np.uint64)
    out_e = np.zeros((N, M, A), np.uint64)
    ndef = np.zeros(N, np.uint64)
    arrs = [np.ascontiguousarray(op_off, np.uint64), np.ascontiguousarray(kind, np.uint8),
            np.ascontiguousarray(actor, np.uint32), np.ascontiguousarray(counter, np.uint64),
            np.ascontiguousarray(rm_row, np.uint32), np.ascontiguousarray(rm_clock, np.uint64),
            np.ascontiguousarray(mem_off, np.uint64), np.ascontiguousarray(mem, np.uint32)]
    t = lib().oracle_orswot_apply_streams(N, M, A, *[_p(a) for a in arrs], _p(out_c), _p(out_e), _p(ndef))
    return out_c, out_e, ndef, t


def bitmap_members(words: np.ndarray) -> frozenset:
    out = []
    for w, x in enumerate(np.asarray(words, dtype=np.uint64).tolist()):
        while x:
            b = (x & -x).bit_length() - 1
            out.append(w * 64 + b)
            x &= x - 1
    return frozenset(out)


# ---------------------------------------------------------------------------------------
# Well-formed ORSWOT replica generator, numpy, for parity at small sizes
# ---------------------------------------------------------------------------------------
def gen_orswot(seed: int, R: int, M: int, A: int, kmax: int = 24, p_def: float = 0.15,
               p_obs_rm: float = 0.25):
    """Dense replicas that keep the reference invariants (each dot unique, e <= c).

    Actor a's k-th event adds member mem(a, k); replica r has seen events 1..c[r, a] of each
    actor; its entry for (m, a) is the latest such event adding m, unless the replica has
    observed a remove of it (prob p_obs_rm).  Some replicas carry deferred removes with a
    future context (rm[a] > c[r, a] for some a) whose effect is pre-applied, as apply_rm
    leaves it (orswot.rs:230-250).
    """
    rng = np.random.default_rng(seed)
    mem = rng.integers(0, M, size=(A, kmax + 1))  # mem[a, k]
    clock = rng.integers(0, kmax + 1, size=(R, A)).astype(np.uint64)
    entries = np.zeros((R, M, A), dtype=np.uint64)
    for r in range(R):
        for a in range(A):
            for k in range(1, int(clock[r, a]) + 1):
                entries[r, mem[a, k], a] = k
    obs = rng.random(size=(R, M, A)) < p_obs_rm
    entries[obs] = 0
    Mw = (M + 63) // 64
    def_off = [0]
    dcl, dmem = [], []
    for r in range(R):
        nd = int(rng.integers(1, 4)) if rng.random() < p_def else 0
        for _ in range(nd):
            rm = clock[r].copy()
            fut = rng.random(A) < 0.1
            fut[rng.integers(0, A)] = True
            rm[fut] += rng.integers(1, 4, size=int(fut.sum())).astype(np.uint64)
            # some removes carry a past (dominated) context on other actors
            back = (rng.random(A) < 0.3) & ~fut
            rm[back] = rm[back] // np.uint64(2)
            ms = rng.choice(M, size=min(M, int(rng.integers(1, 4))), replace=False)
            bits = np.zeros(Mw, dtype=np.uint64)
            for m in ms:
                bits[m // 64] |= np.uint64(1) << np.uint64(m % 64)
                row = entries[r, m]
                row[row <= rm] = 0
            dcl.append(rm)
            dmem.append(bits)
        def_off.append(len(dcl))
    D = len(dcl)
    def_clock = np.array(dcl, dtype=np.uint64).reshape(D, A) if D else np.zeros((0, A), np.uint64)
    def_members = np.array(dmem, dtype=np.uint64).reshape(D, Mw) if D else np.zeros((0, Mw), np.uint64)
    return clock, entries, np.array(def_off, dtype=np.uint64), def_clock, def_members


# ---------------------------------------------------------------------------------------
# Dense restatement of the Orswot lub, checked against the map fold above
# by tests/test_oracle_twins.py; used as the injected local fold in the CPU (gloo) tests.
# ---------------------------------------------------------------------------------------
def dense_orswot_join_fold(clock: np.ndarray, entries: np.ndarray):
    """e = max(e1==e2?e1:0, e1>c2?e1:0, e2>c1?e2:0), c = max(c1,c2), as a left fold."""
    e = np.zeros(entries.shape[1:], dtype=np.uint64)
    c = np.zeros(clock.shape[1], dtype=np.uint64)
    for r in range(entries.shape[0]):
        e2, c2 = entries[r], clock[r]
        t0 = np.where(e == e2, e, 0)
        t1 = np.where(e > c2, e, 0)
        t2 = np.where(e2 > c, e2, 0)
        e = np.maximum(t0, np.maximum(t1, t2)).astype(np.uint64)
        c = np.maximum(c, c2)
    return c, e


def dense_orswot_apply(clock, entries, dcl, dmb, cnt, ops):
    """Dense restatement of one state's Orswot CmRDT::apply stream — the algorithm
    crdt_orswot_apply_batch runs per wave (orswot.rs:55-79, apply_rm :230-250, apply_deferred
    :281-286), checked against Orswot.apply by tests/test_oracle_orswot_apply.py.
    clock (A,), entries (M, A), dcl (Dcap, A), dmb (Dcap, Mw) are updated in place; ops are
    ("add", a, k, members) / ("rm", dense rm row, members).  Returns (deferred count, status)."""
    A = clock.shape[0]
    M = entries.shape[0]
    Dcap = dcl.shape[0]
    st = 0

    def forget(m, rm):  # VClock::forget vclock.rs:95-105 on a dense row
        row = entries[m]
        row[(row != 0) & (row <= rm)] = 0

    def members_of(bits):
        return [m for m in bitmap_members(bits) if m < M]

    for op in ops:
        if op[0] == "add":
            _, a, k, ms = op
            if a >= A:
                st |= 2
                continue
            if clock[a] >= np.uint64(k):  # :60-63
                continue
            for m in ms:  # :65-68
                if m >= M:
                    st |= 2
                    continue
                entries[m, a] = max(entries[m, a], np.uint64(k))
            clock[a] = np.uint64(k)  # :70
            nk = 0  # apply_deferred :281-286
            for d in range(cnt):
                rm = dcl[d].copy()
                for m in members_of(dmb[d]):
                    forget(m, rm)
                if (rm > clock).any():
                    dcl[nk], dmb[nk] = rm, dmb[d].copy()
                    nk += 1
            cnt = nk
        else:
            _, rm, ms = op
            rm = np.asarray(rm, dtype=np.uint64)
            for m in ms:  # :231-238
                if m >= M:
                    st |= 2
                    continue
                forget(m, rm)
            if not (rm > clock).any():  # :239-249, rm <= clock: already seen
                continue
            slot = next((d for d in range(cnt) if np.array_equal(dcl[d], rm)), -1)
            if slot < 0:
                if cnt >= Dcap:
                    st |= 1
                    continue
                slot = cnt
                cnt += 1
                dcl[slot] = rm
                dmb[slot] = 0
            for m in ms:
                if m < M:
                    dmb[slot, m // 64] |= np.uint64(1) << np.uint64(m % 64)
    return cnt, st


def dense_orswot_lub(clock, entries, def_clock, def_members):
    """Join fold, then every deferred remove: forget ceiling on its members, survival
    !(rm <= C), survivors with identical rm clocks merged.  Returns (c, e, deferred set)."""
    c, e = dense_orswot_join_fold(clock, entries)
    surv = {}
    for d in range(def_clock.shape[0]):
        rm = def_clock[d]
        ms = bitmap_members(def_members[d])
        for m in ms:
            e[m] = np.where(e[m] > rm, e[m], 0)
        if np.any(rm > c):
            surv.setdefault(tuple(int(x) for x in rm), set()).update(ms)
    return c, e, {(k, frozenset(v)) for k, v in surv.items()}


def dense_orswot_survivors(final_clock, def_clock, def_members):
    """The deferred part of dense_orswot_lub on whole member bitmaps, given the folded clock:
    a remove survives iff !(rm <= C) (orswot.rs:240-249), survivors with identical rm clocks
    merge their member sets (the HashMap<VClock, HashSet<M>> of :242-246).  Returns the set of
    (rm clock tuple, frozenset members)."""
    c = np.asarray(final_clock, np.uint64)
    surv = {}
    for d in np.flatnonzero(np.any(np.asarray(def_clock, np.uint64) > c[None, :], axis=1)):
        surv.setdefault(tuple(int(x) for x in def_clock[d]), set()).update(bitmap_members(def_members[d]))
    return {(k, frozenset(v)) for k, v in surv.items()}


# ---------------------------------------------------------------------------------------
# Map<u32, MVReg<u64>> (config 4): dense layout, ingest/egress, and the dense restatement
# of the left fold the GPU kernel implements
# ---------------------------------------------------------------------------------------
# Dense replica r of a group (keys, actors and MVReg values interned to indices / u64):
#   clock (R, A); ec (R, K, A) entry clocks (key absent <=> row 0);
#   vclk (R, K, V, A) val clocks, slots in Vec order, empty slot <=> row 0; vval (R, K, V);
#   deferred: def_row (D,) non-decreasing replica index, def_clock (D, A), def_keys (D, Kw).
def _bits(keys, width: int) -> np.ndarray:
    out = np.zeros((width + 63) // 64, dtype=np.uint64)
    for k in keys:
        out[k // 64] |= np.uint64(1) << np.uint64(k % 64)
    return out


def map_to_dense(maps, K: int, A: int, V: int):
    """Ingest Map<int, MVReg<int>> objects with int actors < A and keys < K."""
    R = len(maps)
    clock = np.zeros((R, A), np.uint64)
    ec = np.zeros((R, K, A), np.uint64)
    vclk = np.zeros((R, K, V, A), np.uint64)
    vval = np.zeros((R, K, V), np.uint64)
    def_row, dcl, dk = [], [], []
    for r, m in enumerate(maps):
        for a, c in m.clock.dots.items():
            clock[r, a] = c
        for k, e in m.entries.items():
            for a, c in e.clock.dots.items():
                ec[r, k, a] = c
            if len(e.val.vals) > V:
                raise ValueError(f"replica {r} key {k}: {len(e.val.vals)} vals > V={V}")
            for s, (c, v) in enumerate(e.val.vals):
                for a, x in c.dots.items():
                    vclk[r, k, s, a] = x
                vval[r, k, s] = v
        for rm, keys in m.deferred.items():
            row = np.zeros(A, np.uint64)
            for a, c in rm.dots.items():
                row[a] = c
            def_row.append(r)
            dcl.append(row)
            dk.append(_bits(keys, K))
    D = len(def_row)
    Kw = (K + 63) // 64
    return dict(clock=clock, ec=ec, vclk=vclk, vval=vval,
                def_row=np.array(def_row, np.uint64),
                def_clock=np.array(dcl, np.uint64).reshape(D, A),
                def_keys=np.array(dk, np.uint64).reshape(D, Kw))


def _vc_row(row) -> VClock:
    return VClock({a: int(c) for a, c in enumerate(np.asarray(row).tolist()) if c})


def dense_to_map(clock, ec, vclk, vval, deferred=()) -> Map:
    """Egress of one folded dense state (clock (A,), ec (K,A), vclk (K,V,A), vval (K,V))."""
    m = Map(MVReg)
    m.clock = _vc_row(clock)
    for k in range(ec.shape[0]):
        if not ec[k].any():
            continue
        vals = [(_vc_row(vclk[k, s]), int(vval[k, s])) for s in range(vclk.shape[1]) if vclk[k, s].any()]
        m.entries[k] = MapEntry(_vc_row(ec[k]), MVReg(vals))
    for rm, keys in deferred:
        m.deferred[_vc_row(rm)] = set(keys)
    return m


def map_fold_objects(maps) -> Map:
    """The reference left fold: acc = Map::new(); for r: acc.merge(r)."""
    acc = Map(maps[0].vnew if maps else MVReg)
    for m in maps:
        acc.merge(m)
    return acc


def _forget_vals(vals, x):
    out = []
    for c, v in vals:
        c = np.where(c > x, c, np.uint64(0)).astype(np.uint64)
        if c.any():
            out.append((c, v))
    return out


def _lt(x, y) -> bool:  # VClock partial_cmp == Less on dense rows
    return bool(np.all(x <= y) and np.any(x != y))


def _mv_merge(s, o):  # mvreg.rs:112-128 on dense rows
    s = [(c, v) for c, v in s if not any(_lt(c, c2) for c2, _ in o)]
    add = [(c, v) for c, v in o if not any(_lt(c, c1) for c1, _ in s)
           and all(np.any(c != c1) for c1, _ in s)]
    return s + add


def map_drop_steps(clock, def_row, def_clock):
    """t[d]: the step of the fold after which deferred remove d leaves acc.deferred — the first
    i >= def_row[d] with max(clock[0..=i]) >= rm (R if never, i.e. it survives the fold).
    Within [def_row[d], t[d]] it forgets its keys at every step (map.rs:213-219, :311-348)."""
    R, A = clock.shape
    P = np.zeros((R + 1, A), np.uint64)
    for i in range(R):
        P[i + 1] = np.maximum(P[i], clock[i])
    t = []
    for j, rm in zip(np.asarray(def_row).tolist(), def_clock):
        i = int(j)
        while i < R and not np.all(P[i + 1] >= rm):
            i += 1
        t.append(i)
    return np.array(t, np.int64), P


def dense_map_fold(clock, ec, vclk, vval, def_row, def_clock, def_keys, Vout: int):
    """Dense restatement of the Map<K, MVReg> left fold, key by key (keys are independent
    given the replica clocks and the deferred list).  Per step i and key k:
      1. the entry join of map.rs:142-210 with Cs = max(clock[0..i)) and Co = clock[i];
      2. every deferred remove active at step i (def_row <= i <= t) that names k forgets the
         entry (map.rs:213-215 + :311-348; successive forgets compose to one by their max).
    Returns (clock (A,), ec (K,A), vclk (K,Vout,A), vval (K,Vout), nval (K,), deferred set)."""
    R, K, A = ec.shape
    V = vclk.shape[2]
    t, P = map_drop_steps(clock, def_row, def_clock)
    rows = np.asarray(def_row, np.int64)
    o_ec = np.zeros((K, A), np.uint64)
    o_vc = np.zeros((K, Vout, A), np.uint64)
    o_vv = np.zeros((K, Vout), np.uint64)
    o_n = np.zeros(K, np.int64)
    z = np.uint64(0)
    for k in range(K):
        kb = [d for d in range(len(rows)) if (int(def_keys[d][k // 64]) >> (k % 64)) & 1]
        present, e, vals = False, np.zeros(A, np.uint64), []
        for i in range(R):
            Cs, Co = P[i], clock[i]
            e2 = ec[i, k]
            p2 = bool(e2.any())
            if present and not p2:  # :146-161
                if np.all(Co >= e):
                    present, e, vals = False, np.zeros(A, np.uint64), []
                else:
                    e = np.where(e > Co, e, z).astype(np.uint64)
                    vals = _forget_vals(vals, np.where(Co > e, Co, z))
            elif p2 and not present:  # :193-208
                if not np.all(Cs >= e2):
                    e = np.where(e2 > Cs, e2, z).astype(np.uint64)
                    v2 = [(vclk[i, k, s].copy(), int(vval[i, k, s])) for s in range(V) if vclk[i, k, s].any()]
                    vals = _forget_vals(v2, np.where(Cs > e, Cs, z))
                    present = True
            elif present and p2:  # :170-192
                common = np.maximum(np.where(e == e2, e, z),
                                    np.maximum(np.where(e2 > Cs, e2, z), np.where(e > Co, e, z)))
                if not common.any():
                    present, e, vals = False, np.zeros(A, np.uint64), []
                else:
                    v2 = [(vclk[i, k, s].copy(), int(vval[i, k, s])) for s in range(V) if vclk[i, k, s].any()]
                    vals = _mv_merge(vals, v2)
                    dl = np.maximum(e, e2)
                    vals = _forget_vals(vals, np.where(dl > common, dl, z))
                    e = common.astype(np.uint64)
            act = [d for d in kb if rows[d] <= i <= t[d]]
            if act and present:
                ceil = np.max(np.stack([def_clock[d] for d in act]), axis=0)
                e = np.where(e > ceil, e, z).astype(np.uint64)
                if not e.any():
                    present, vals = False, []
                else:
                    vals = _forget_vals(vals, ceil)
        if present:
            o_ec[k] = e
            o_n[k] = len(vals)
            for s, (c, v) in enumerate(vals[:Vout]):
                o_vc[k, s] = c
                o_vv[k, s] = v
    surv = {}
    for d in range(len(rows)):
        if t[d] == R:
            keys = {k for k in range(K) if (int(def_keys[d][k // 64]) >> (k % 64)) & 1}
            surv.setdefault(tuple(int(x) for x in def_clock[d]), set()).update(keys)
    deferred = {(c, frozenset(ks)) for c, ks in surv.items()}
    return P[R].copy(), o_ec, o_vc, o_vv, o_n, deferred


def map_fold(clock, ec, vclk, vval, def_row=None, def_clock=None, def_keys=None, Vout: int = 4,
             peak: Optional[np.ndarray] = None, threads: Optional[int] = None):
    """C++ twin (ref_fold.cpp oracle_map_fold): the reference fold over map-based states.
    Returns (clock, ec, vclk, vval, nval, deferred set, fold seconds); `peak` (K,) u64, if
    given, receives the most values each key held after any step's entry join.  `threads`: the
    multi-core baseline (oracle_map_fold_mt: key ranges per thread, every replica; same result)."""
    clock, ec, vclk, vval = _c64(clock), _c64(ec), _c64(vclk), _c64(vval)
    R, K, A = ec.shape
    V = vclk.shape[2]
    Kw = (K + 63) // 64
    if def_row is None or len(def_row) == 0:
        def_off = np.zeros(R + 1, np.uint64)
        def_clock = np.zeros((1, A), np.uint64)
        def_keys = np.zeros((1, Kw), np.uint64)
        D = 0
    else:
        rows = np.asarray(def_row, np.int64)
        assert np.all(np.diff(rows) >= 0), "def_row must be non-decreasing"
        def_off = np.searchsorted(rows, np.arange(R + 1), side="left").astype(np.uint64)
        D = len(rows)
    def_clock, def_keys = _c64(def_clock), _c64(def_keys)
    maxd = max(D, 1)
    oc = np.zeros(A, np.uint64)
    oe = np.zeros((K, A), np.uint64)
    ovc = np.zeros((K, Vout, A), np.uint64)
    ovv = np.zeros((K, Vout), np.uint64)
    on = np.zeros(K, np.uint64)
    odc = np.zeros((maxd, A), np.uint64)
    odk = np.zeros((maxd, Kw), np.uint64)
    nd = ctypes.c_size_t(0)
    if threads is None:
        t = lib().oracle_map_fold(_p(clock), _p(ec), _p(vclk), _p(vval), R, K, A, V, _p(def_off),
                                  _p(def_clock), _p(def_keys), Vout, _p(oc), _p(oe), _p(ovc), _p(ovv),
                                  _p(on), _p(odc), _p(odk), maxd, ctypes.byref(nd),
                                  _p(peak) if peak is not None else None)
    else:
        assert peak is None, "map_fold: peak is single-threaded instrumentation"
        t = lib().oracle_map_fold_mt(_p(clock), _p(ec), _p(vclk), _p(vval), R, K, A, V, _p(def_off),
                                     _p(def_clock), _p(def_keys), Vout, int(threads), _p(oc), _p(oe), _p(ovc),
                                     _p(ovv), _p(on), _p(odc), _p(odk), maxd, ctypes.byref(nd))
    n = nd.value
    assert n <= maxd
    deferred = {(tuple(int(x) for x in odc[k]), bitmap_members(odk[k])) for k in range(n)}
    return oc, oe, ovc, ovv, on.astype(np.int64), deferred, t


def gen_map_replicas(seed: int, R: int, K: int, A: int, steps: int = 200, p_ooo: float = 0.4,
                     p_up: float = 0.4, p_rm: float = 0.15, vnew=None, write=None):
    """Realistic Map<int, MVReg<int>> replica states by op replay (reference semantics).

    A actors each own a replica and, at random: write a key (ctx from get(key), map.rs:272,
    test/map.rs:71-125), remove a key (rm ctx from get(key), test/map.rs:127-146), deliver
    logged ops of other actors (out of causal order with prob p_ooo — which is what leaves
    deferred removes, test/map.rs:265-300), or merge another actor's state (gossip).  R
    snapshots of actor states at random times are returned (the fold's replicas).  `vnew` /
    `write(value, ctx, val, actor) -> value op` select another value type (default MVReg::write)."""
    rng = np.random.default_rng(seed)
    vnew = vnew or MVReg
    write = write or (lambda r, c, v, a: r.write(v, c))
    reps = [Map(vnew) for _ in range(A)]
    seen = [set() for _ in range(A)]
    log = []
    snaps = []
    val = 1
    for step in range(steps):
        a = int(rng.integers(A))
        m = reps[a]
        x = rng.random()
        if x < p_up:
            k = int(rng.integers(K))
            op = m.update(k, m.get(k).derive_add_ctx(a), lambda r, c, v=val, a=a: write(r, c, v, a))
            val += 1
            m.apply(op)
            seen[a].add(len(log))
            log.append(op)
        elif x < p_up + p_rm:
            k = int(rng.integers(K))
            # the rm ctx is read at this replica, or (a client that read elsewhere) at another
            # replica whose context this one may not have seen yet -> a deferred remove
            src = m if rng.random() < 0.5 else reps[int(rng.integers(A))]
            op = m.rm(k, src.get(k).derive_rm_ctx())
            m.apply(op)
            seen[a].add(len(log))
            log.append(op)
        elif x < p_up + p_rm + 0.25 and log:
            todo = [i for i in range(len(log)) if i not in seen[a]]
            if todo:
                if rng.random() < p_ooo:
                    todo = list(rng.permutation(todo))
                for i in todo[: int(rng.integers(1, 4))]:
                    m.apply(log[int(i)])
                    seen[a].add(int(i))
        else:
            b = int(rng.integers(A))
            if b != a:
                m.merge(reps[b])
                seen[a] |= seen[b]
        if rng.random() < R / steps * 1.5 and len(snaps) < R:
            snaps.append(m.copy())
    while len(snaps) < R:
        snaps.append(reps[int(rng.integers(A))].copy())
    order = rng.permutation(R)
    return [snaps[int(i)] for i in order]


# ---- Map<K, GCounter> / Map<K, PNCounter> (counter values, round 4) ------------------------------
def counter_rows(val, A: int) -> np.ndarray:
    """The dense value rows of a counter: GCounter -> (1, A), PNCounter -> (2, A) [P, N]."""
    parts = [val.inner] if isinstance(val, GCounter) else [val.p.inner, val.n.inner]
    out = np.zeros((len(parts), A), np.uint64)
    for w, vc in enumerate(parts):
        for a, c in vc.dots.items():
            out[w, a] = c
    return out


def counter_from_rows(rows, W: int):
    if W == 1:
        g = GCounter()
        g.inner = _vc_row(rows[0])
        return g
    c = PNCounter()
    c.p.inner, c.n.inner = _vc_row(rows[0]), _vc_row(rows[1])
    return c


def map_counter_to_dense(maps, K: int, A: int, W: int):
    """Ingest Map<int, GCounter> (W = 1) or Map<int, PNCounter> (W = 2) objects: clock (R, A),
    ec (R, K, A), val (R, K, W, A) and the deferred pool (def_row, def_clock, def_keys)."""
    R = len(maps)
    clock = np.zeros((R, A), np.uint64)
    ec = np.zeros((R, K, A), np.uint64)
    val = np.zeros((R, K, W, A), np.uint64)
    def_row, dcl, dk = [], [], []
    for r, m in enumerate(maps):
        for a, c in m.clock.dots.items():
            clock[r, a] = c
        for k, e in m.entries.items():
            for a, c in e.clock.dots.items():
                ec[r, k, a] = c
            val[r, k] = counter_rows(e.val, A)
        for rm, keys in m.deferred.items():
            row = np.zeros(A, np.uint64)
            for a, c in rm.dots.items():
                row[a] = c
            def_row.append(r)
            dcl.append(row)
            dk.append(_bits(keys, K))
    D = len(def_row)
    Kw = (K + 63) // 64
    return dict(clock=clock, ec=ec, val=val, def_row=np.array(def_row, np.uint64),
                def_clock=np.array(dcl, np.uint64).reshape(D, A), def_keys=np.array(dk, np.uint64).reshape(D, Kw))


def dense_to_map_counter(clock, ec, val, deferred=()) -> Map:
    """Egress of one folded dense Map<K, counter> state (clock (A,), ec (K, A), val (K, W, A))."""
    W = val.shape[1]
    m = Map(GCounter if W == 1 else PNCounter)
    m.clock = _vc_row(clock)
    for k in range(ec.shape[0]):
        if ec[k].any():
            m.entries[k] = MapEntry(_vc_row(ec[k]), counter_from_rows(val[k], W))
    for rm, keys in deferred:
        m.deferred[_vc_row(rm)] = set(keys)
    return m


def map_counter_objects(R: int, K: int, A: int, W: int, seed: int, steps: int = 300, **kw):
    """Op-replay replicas of Map<int, GCounter> (W = 1: every write an inc of the writer's dot)
    or Map<int, PNCounter> (W = 2: inc or dec at random)."""
    rng = np.random.default_rng(seed ^ 0x6C0)
    if W == 1:
        return gen_map_replicas(seed, R, K, A, steps=steps, vnew=GCounter, write=lambda v, c, x, a: v.inc(a), **kw)
    return gen_map_replicas(seed, R, K, A, steps=steps, vnew=PNCounter,
                            write=lambda v, c, x, a: v.inc(a) if rng.random() < 0.6 else v.dec(a), **kw)


# ---- Map<K, Orswot<M>> (nested Orswot values, round 4; the reference's merge_error KAT type) -------
def map_orswot_to_dense(maps, K: int, M: int, A: int):
    """Ingest Map<int, Orswot<int>> objects (keys < K, members < M, actors < A): clock (R, A),
    ec (R, K, A), oc (R, K, A) the nested Orswot clocks, ent (R, K, M, A) its member dots, the
    nested deferred removes as a CSR over (replica, key) — vd_off (R*K + 1), vd_clock (Dv, A),
    vd_members (Dv,) member bitmasks ((Dv, Mw) words past M = 64) — and the Map's own deferred pool
    (def_row, def_clock, def_keys)."""
    Mw = max(1, (M + 63) // 64)
    R = len(maps)
    clock = np.zeros((R, A), np.uint64)
    ec = np.zeros((R, K, A), np.uint64)
    oc = np.zeros((R, K, A), np.uint64)
    ent = np.zeros((R, K, M, A), np.uint64)
    vd_off, vdc, vdm = [0], [], []
    def_row, dcl, dk = [], [], []
    for r, m in enumerate(maps):
        for a, c in m.clock.dots.items():
            clock[r, a] = c
        for k in range(K):
            e = m.entries.get(k)
            if e is not None:
                for a, c in e.clock.dots.items():
                    ec[r, k, a] = c
                for a, c in e.val.clock.dots.items():
                    oc[r, k, a] = c
                for mem, mc in e.val.entries.items():
                    for a, c in mc.dots.items():
                        ent[r, k, mem, a] = c
                for rm, mems in e.val.deferred.items():
                    row = np.zeros(A, np.uint64)
                    for a, c in rm.dots.items():
                        row[a] = c
                    vdc.append(row)
                    vdm.append(int(_bits(mems, 64)[0]) if Mw == 1 else _bits(mems, 64 * Mw))
            vd_off.append(len(vdc))
        for rm, keys in m.deferred.items():
            row = np.zeros(A, np.uint64)
            for a, c in rm.dots.items():
                row[a] = c
            def_row.append(r)
            dcl.append(row)
            dk.append(_bits(keys, K))
    D, Dv = len(def_row), len(vdc)
    Kw = (K + 63) // 64
    return dict(clock=clock, ec=ec, oc=oc, ent=ent, vd_off=np.array(vd_off, np.uint64),
                vd_clock=np.array(vdc, np.uint64).reshape(Dv, A), vd_members=np.array(vdm, np.uint64).reshape((Dv,) if Mw == 1 else (Dv, Mw)),
                def_row=np.array(def_row, np.uint64), def_clock=np.array(dcl, np.uint64).reshape(D, A),
                def_keys=np.array(dk, np.uint64).reshape(D, Kw))


def dense_to_map_orswot(clock, ec, oc, ent, vdeferred=None, deferred=()) -> Map:
    """Egress of one folded dense Map<K, Orswot> state: clock (A,), ec / oc (K, A), ent (K, M, A),
    vdeferred {key: [(rm row, member set)]}, deferred [(rm row, key set)]."""
    m = Map(Orswot)
    m.clock = _vc_row(clock)
    for k in range(ec.shape[0]):
        if ec[k].any():
            o = Orswot()
            o.clock = _vc_row(oc[k])
            for mem in range(ent.shape[1]):
                if ent[k, mem].any():
                    o.entries[mem] = _vc_row(ent[k, mem])
            for rm, mems in (vdeferred or {}).get(k, []):
                o.deferred[_vc_row(rm)] = set(mems)
            m.entries[k] = MapEntry(_vc_row(ec[k]), o)
    for rm, keys in deferred:
        m.deferred[_vc_row(rm)] = set(keys)
    return m


def map_orswot_objects(R: int, K: int, M: int, A: int, seed: int, steps: int = 300, p_vrm: float = 0.35, **kw):
    """Op-replay replicas of Map<int, Orswot<int>>: a write adds a member under the Map's dot, or
    (p_vrm) removes one with the nested Orswot's contains() context (test/map.rs's nested-set
    pattern), so out-of-order delivery leaves deferred removes at both levels."""
    rng = np.random.default_rng(seed ^ 0x0E5)

    def write(v, c, x, a):
        mem = int(rng.integers(M))
        if rng.random() < p_vrm:
            ctx = v.contains(mem).derive_rm_ctx()
            if rng.random() < 0.5:  # a context read at a replica that has seen more adds: deferred
                b = int(rng.integers(A))
                ctx.clock.apply(Dot(b, ctx.clock.get(b) + int(rng.integers(1, 3))))
            return v.rm(mem, ctx)
        return v.add(mem, c)
    return gen_map_replicas(seed, R, K, A, steps=steps, vnew=Orswot, write=write, **kw)


# ---- Map<K, Map<K2, MVReg<int>>> (the reference's own Map test type TMap, test/map.rs:10; round 5) ----
def nested_map_to_dense(maps, K: int, K2: int, A: int, V: int):
    """Ingest Map<int, Map<int, MVReg<int>>> objects (outer keys < K, inner keys < K2 <= 256, actors < A,
    at most V values per register): clock (R, A), ec / ic (R, K, A) the outer entry / inner Map clocks,
    iec (R, K, K2, A), ivc (R, K, K2, V, A) / ivv (R, K, K2, V) the MVReg slots in Vec order, the inner
    deferred removes as a CSR over (replica, key) — id_off (R*K + 1), id_clock (Di, A), id_keys (Di,)
    inner-key bitmasks ((Di, ceil(K2/64)) words past K2 = 64) — and the outer deferred pool (def_row,
    def_clock, def_keys)."""
    R = len(maps)
    clock = np.zeros((R, A), np.uint64)
    ec = np.zeros((R, K, A), np.uint64)
    ic = np.zeros((R, K, A), np.uint64)
    iec = np.zeros((R, K, K2, A), np.uint64)
    ivc = np.zeros((R, K, K2, V, A), np.uint64)
    ivv = np.zeros((R, K, K2, V), np.uint64)
    id_off, idc, idk = [0], [], []
    def_row, dcl, dk = [], [], []

    def row(vc):
        out = np.zeros(A, np.uint64)
        for a, c in vc.dots.items():
            out[a] = c
        return out

    for r, m in enumerate(maps):
        clock[r] = row(m.clock)
        for k in range(K):
            e = m.entries.get(k)
            if e is not None:
                ec[r, k] = row(e.clock)
                ic[r, k] = row(e.val.clock)
                for j, ie in e.val.entries.items():
                    iec[r, k, j] = row(ie.clock)
                    assert len(ie.val.vals) <= V, "more values than V slots"
                    for s, (vcl, x) in enumerate(ie.val.vals):
                        ivc[r, k, j, s] = row(vcl)
                        ivv[r, k, j, s] = x
                for rm, keys in e.val.deferred.items():
                    idc.append(row(rm))
                    idk.append(_bits(keys, max(K2, 64)))
            id_off.append(len(idc))
        for rm, keys in m.deferred.items():
            def_row.append(r)
            dcl.append(row(rm))
            dk.append(_bits(keys, K))
    D, Di = len(def_row), len(idc)
    Kw = (K + 63) // 64
    return dict(clock=clock, ec=ec, ic=ic, iec=iec, ivc=ivc, ivv=ivv, id_off=np.array(id_off, np.uint64),
                id_clock=np.array(idc, np.uint64).reshape(Di, A),
                id_keys=(np.array(idk, np.uint64).reshape(Di, max(K2, 64) // 64 if K2 <= 64 else (K2 + 63) // 64)
                         if K2 > 64 else np.array([int(x[0]) for x in idk], np.uint64)),
                def_row=np.array(def_row, np.uint64), def_clock=np.array(dcl, np.uint64).reshape(D, A),
                def_keys=np.array(dk, np.uint64).reshape(D, Kw))


def dense_to_nested_map(clock, ec, ic, iec, ivc, ivv, nval, ideferred=None, deferred=()) -> Map:
    """Egress of one folded dense nested Map state: clock (A,), ec / ic (K, A), iec (K, K2, A), ivc (K,
    K2, S, A) / ivv (K, K2, S) with nval (K, K2) slots used, ideferred {key: [(rm row, key set)]},
    deferred [(rm row, key set)]."""
    m = Map(lambda: Map(MVReg))
    m.clock = _vc_row(clock)
    for k in range(ec.shape[0]):
        if ec[k].any():
            inner = Map(MVReg)
            inner.clock = _vc_row(ic[k])
            for j in range(iec.shape[1]):
                if iec[k, j].any():
                    reg = MVReg()
                    reg.vals = [(_vc_row(ivc[k, j, s]), int(ivv[k, j, s])) for s in range(int(nval[k, j]))]
                    inner.entries[j] = MapEntry(_vc_row(iec[k, j]), reg)
            for rm, keys in (ideferred or {}).get(k, []):
                inner.deferred[_vc_row(rm)] = set(keys)
            m.entries[k] = MapEntry(_vc_row(ec[k]), inner)
    for rm, keys in deferred:
        m.deferred[_vc_row(rm)] = set(keys)
    return m


def nested_map_objects(R: int, K: int, K2: int, A: int, seed: int, steps: int = 300, p_irm: float = 0.3, **kw):
    """Op-replay replicas of Map<int, Map<int, MVReg<int>>>: a write updates the outer key with an inner
    write (inner.update(k2, ctx, reg.write)) or (p_irm) an inner remove whose context is read at the
    inner Map — sometimes at a replica that has seen more (a deferred inner remove), as test/map.rs's
    build_ops mixes inner Up / Rm under one outer dot."""
    rng = np.random.default_rng(seed ^ 0x4E5)

    def write(v, c, x, a):
        j = int(rng.integers(K2))
        if rng.random() < p_irm:
            ctx = v.get(j).derive_rm_ctx()
            if rng.random() < 0.5:
                b = int(rng.integers(A))
                ctx.clock.apply(Dot(b, ctx.clock.get(b) + int(rng.integers(1, 3))))
            return v.rm(j, ctx)
        return v.update(j, c, lambda reg, cx, x=x: reg.write(x, cx))
    return gen_map_replicas(seed, R, K, A, steps=steps, vnew=lambda: Map(MVReg), write=write, **kw)


def max_vals(maps) -> int:
    return max([len(e.val.vals) for m in maps for e in m.entries.values()] + [1])


# ---------------------------------------------------------------------------------------
# Well-formed synthetic Map<K, MVReg<u64>> replicas (config 4): numpy restatement of
# rust-crdt_amd/csrc/synth.hip crdt_synth_map (bit-exact), used for sampled-key parity.
# ---------------------------------------------------------------------------------------
_SALT_KIND = np.uint64(0xA5A5A5A55A5A5A5A)
_SALT_VAL = np.uint64(0x5EED5EED0B57AC1E)
_SALT_DEF = np.uint64(0xDEF0DEF0DEF0DEF0)


def _key_count(K: int, A: int, res: int) -> int:
    """#{k < K : k % A == res}."""
    return (K - res + A - 1) // A if res < K else 0


def map_keys_of(a: int, K: int, A: int) -> np.ndarray:
    """The keys actor a writes, in its round-robin order: k % A == a, then k % A == a-1."""
    if A == 1:
        return np.arange(K, dtype=np.int64)
    prim = np.arange(a, K, A, dtype=np.int64)
    sec = np.arange((a - 1) % A, K, A, dtype=np.int64)
    return np.concatenate([prim, sec])


def synth_map_clock(seed: int, rows: int, A: int, kmax: int, row0: int = 0) -> np.ndarray:
    r = np.arange(row0, row0 + rows, dtype=np.uint64)
    a = np.arange(A, dtype=np.uint64)
    with np.errstate(over="ignore"):
        c = mix64(np.uint64(seed) + (r[:, None] * np.uint64(A) + a[None, :] + np.uint64(1)) * _GOLD)
    return (c % np.uint64(kmax + 1)).astype(np.uint64)


def _op_hash(seed: int, salt, a, n):
    with np.errstate(over="ignore"):
        return mix64((np.uint64(seed) ^ salt) + (np.asarray(a, np.uint64) << np.uint64(32)) + np.asarray(n, np.uint64))


def synth_map_deferred(seed: int, rows: int, K: int, A: int, kmax: int, p_def: float = 0.1,
                       row0: int = 0):
    """Deferred removes with a future context, per replica (closed form in the replica index,
    so every rank of a sharded run builds the same global list).  Returns (def_row local,
    def_clock (D, A), def_keys (D, Kw))."""
    c = synth_map_clock(seed, rows, A, kmax, row0)
    Kw = (K + 63) // 64
    rows_out, dcl, dk = [], [], []
    thr = int(p_def * 1000)
    for rl in range(rows):
        with np.errstate(over="ignore"):
            h = int(mix64((np.uint64(seed) ^ _SALT_DEF) + np.uint64(row0 + rl)))
        nd = 1 + (h >> 32) % 2 if h % 1000 < thr else 0
        for d in range(nd):
            hd = int(mix64(np.uint64((h + 0x9E37 * (d + 1)) & (2**64 - 1))))
            w = hd % A
            rm = np.zeros(A, np.uint64)
            rm[w] = c[rl, w] + np.uint64(1 + (hd >> 8) % 4)
            if A > 1:
                b = (w + 1 + (hd >> 16) % (A - 1)) % A
                rm[b] = c[rl, b] // np.uint64(2)
            keys = map_keys_of(w, K, A)
            bits = np.zeros(Kw, np.uint64)
            for i in range(1 + (hd >> 24) % 3):
                j = int(mix64(np.uint64((hd + i + 1) & (2**64 - 1)))) % len(keys)
                k = int(keys[j])
                bits[k // 64] |= np.uint64(1) << np.uint64(k % 64)
            rows_out.append(rl)
            dcl.append(rm)
            dk.append(bits)
    D = len(rows_out)
    return (np.array(rows_out, np.int64), np.array(dcl, np.uint64).reshape(D, A),
            np.array(dk, np.uint64).reshape(D, Kw))


def synth_map(seed: int, rows: int, K: int, A: int, V: int, kmax: int, row0: int = 0,
              keys=None, deferred=None, clock_override=None):
    """Dense replicas [row0, row0+rows) for the key subset `keys` (default all).

    Model (every replica is a causally closed state of one op history): key k is written by
    actors w0 = k % A and w1 = (k+1) % A; actor a's n-th op (n = 1, 2, ...) targets the
    ((n-1) mod M_a)-th key of map_keys_of(a) and is a remove (1/8, mix of (a, n)) or an update
    writing val mix(a, n) with MVReg clock {a: n} (derive_add_ctx of a state that has seen only
    a's own ops, map.rs:272, ctx.rs:42-48).  Replica r has seen ops 1..c[r][a] of every actor.
    So entry (r, k) holds, per writer w in (w0, w1) order, w's latest op on k if it is an
    update: ec[w] = n, one MVReg value ({w: n}, mix(w, n)); a remove (rm clock = w's own entry
    view, map.rs:291) leaves nothing of w.  Deferred removes (synth_map_deferred) of the replica
    are pre-applied (apply_keyset_rm, map.rs:318-333): a writer's dot survives iff n > rm[w]."""
    keys = np.arange(K, dtype=np.int64) if keys is None else np.asarray(keys, np.int64)
    c = synth_map_clock(seed, rows, A, kmax, row0) if clock_override is None else np.asarray(clock_override, np.uint64)
    nk = len(keys)
    ec = np.zeros((rows, nk, A), np.uint64)
    vclk = np.zeros((rows, nk, V, A), np.uint64)
    vval = np.zeros((rows, nk, V), np.uint64)
    ceil = np.zeros((rows, nk, A), np.uint64)
    if deferred is not None:
        drow, dcl, dk = deferred
        pos = {int(k): i for i, k in enumerate(keys)}
        for d in range(len(drow)):
            for k in bitmap_members(dk[d]):
                if k in pos:
                    i = pos[k]
                    ceil[drow[d], i] = np.maximum(ceil[drow[d], i], dcl[d])
    writers = [0] if A == 1 else [0, 1]
    slot = np.zeros((rows, nk), np.int64)
    for wi in writers:
        w = (keys + wi) % A
        if A == 1:
            M = np.full(nk, K, np.int64)
            j = keys.copy()
        else:
            P = np.array([_key_count(K, A, int(x)) for x in w], np.int64)
            S = np.array([_key_count(K, A, int((x - 1) % A)) for x in w], np.int64)
            M = P + S
            j = np.where(keys % A == w, keys // A, P + keys // A)
        cw = c[:, w].astype(np.int64)  # (rows, nk)
        n = np.where(cw >= j[None] + 1, j[None] + 1 + M[None] * ((cw - j[None] - 1) // M[None]), 0)
        isrm = (_op_hash(seed, _SALT_KIND, w[None].astype(np.uint64), n.astype(np.uint64)) & np.uint64(7)) == 0
        val = _op_hash(seed, _SALT_VAL, w[None].astype(np.uint64), n.astype(np.uint64))
        cl = np.take_along_axis(ceil, np.broadcast_to(w[None, :, None], (rows, nk, 1)), axis=2)[..., 0]
        live = (n > 0) & ~isrm & (n.astype(np.uint64) > cl)
        rr, kk = np.nonzero(live)
        ww = w[kk]
        ec[rr, kk, ww] = n[rr, kk].astype(np.uint64)
        s = slot[rr, kk]
        ok = s < V
        vclk[rr[ok], kk[ok], s[ok], ww[ok]] = n[rr, kk][ok].astype(np.uint64)
        vval[rr[ok], kk[ok], s[ok]] = val[rr, kk][ok]
        slot[rr, kk] += 1
    return dict(clock=c, ec=ec, vclk=vclk, vval=vval)


def restrict_deferred_keys(def_keys: np.ndarray, keys) -> np.ndarray:
    """Re-index key bitmaps onto a key subset (keys[i] -> bit i); keys are independent in the
    Map fold given the clocks, so folding a key subset restricts the full fold exactly."""
    keys = np.asarray(keys, np.int64)
    out = np.zeros((def_keys.shape[0], (len(keys) + 63) // 64), np.uint64)
    for i, k in enumerate(keys.tolist()):
        bit = (def_keys[:, k // 64] >> np.uint64(k % 64)) & np.uint64(1)
        out[:, i // 64] |= bit << np.uint64(i % 64)
    return out


# ---------------------------------------------------------------------------------------
# bincode 1.x (default options) restatement of the serde derives, used by
# tests/test_*wire*.py to build and check the frames crdt_*_ingest / _egress read and write.
# Published encoding: little-endian fixed-width integers; a struct is its fields in order; a
# map / set / Vec is a u64 length then its entries (key, value).  The reference types'
# derives: VClock { dots: BTreeMap<A, u64> } (vclock.rs:56-60), GCounter { inner } (gcounter.rs:25-28),
# PNCounter { p, n } (pncounter.rs:28-32), GSet { value: BTreeSet } (gset.rs:7-10),
# LWWReg { val, marker } (lwwreg.rs:13-19), Orswot { clock, entries: HashMap<M, VClock>,
# deferred: HashMap<VClock, HashSet<M>> } (orswot.rs:20-25), Map { clock, entries: BTreeMap<K,
# Entry { clock, val }>, deferred: HashMap<VClock, BTreeSet<K>> } (map.rs:31-47) with
# MVReg { vals: Vec<(VClock, V)> } (mvreg.rs:32-35).  Actors u32, members / elements u64, Map keys
# u32, MVReg values u64 (BASELINE config 4's Map<u32, MVReg<u64>>).
# Parity of the byte format itself is unpinned (the reference ships no serialized fixtures and
# bincode is not among its dependencies); the semantic round trips are pinned by the KATs.
# ---------------------------------------------------------------------------------------
import struct as _st


def bc_vclock(dots) -> bytes:
    items = sorted((int(a), int(c)) for a, c in dict(dots).items() if c)
    return _st.pack("<Q", len(items)) + b"".join(_st.pack("<IQ", a, c) for a, c in items)


def bc_pncounter(p, n) -> bytes:
    return bc_vclock(p) + bc_vclock(n)


def bc_gset(values) -> bytes:
    v = sorted(int(x) for x in values)
    return _st.pack("<Q", len(v)) + b"".join(_st.pack("<Q", x) for x in v)


def bc_lwwreg(val, marker) -> bytes:
    return _st.pack("<QQ", int(val), int(marker))


def bc_orswot(clock, entries, deferred, order=None) -> bytes:
    """clock {a: c}; entries {m: {a: c}}; deferred [(rm {a: c}, members)].  `order` (optional)
    permutes the entries (a HashMap serializes in any order)."""
    ms = list(entries) if order is None else order
    out = bc_vclock(clock) + _st.pack("<Q", len(ms))
    for m in ms:
        out += _st.pack("<Q", int(m)) + bc_vclock(entries[m])
    out += _st.pack("<Q", len(deferred))
    for rm, members in deferred:
        mem = list(members)
        out += bc_vclock(rm) + _st.pack("<Q", len(mem)) + b"".join(_st.pack("<Q", int(x)) for x in mem)
    return out


def bc_map(clock, entries, deferred, key_order=None) -> bytes:
    """Map<u32, MVReg<u64, u32>, u32> (map.rs:31-47, mvreg.rs:32-35): clock {a: c}; entries
    {k: (entry clock {a: c}, [(value clock {a: c}, val), ...] in Vec order)}, serialized in key
    order (BTreeMap); deferred [(rm {a: c}, keys)] (HashMap<VClock, BTreeSet<K>>: keys ascending)."""
    ks = sorted(entries) if key_order is None else key_order
    out = bc_vclock(clock) + _st.pack("<Q", len(ks))
    for k in ks:
        ec, vals = entries[k]
        out += _st.pack("<I", int(k)) + bc_vclock(ec) + _st.pack("<Q", len(vals))
        for vc, v in vals:
            out += bc_vclock(vc) + _st.pack("<Q", int(v))
    out += _st.pack("<Q", len(deferred))
    for rm, keys in deferred:
        kk = sorted(int(x) for x in keys)
        out += bc_vclock(rm) + _st.pack("<Q", len(kk)) + b"".join(_st.pack("<I", x) for x in kk)
    return out


def unbc_map(b: bytes, pos: int = 0):
    """-> (clock, entries {k: (dots, [(dots, val)])}, deferred {tuple(sorted rm items): set(keys)}, pos)."""
    clock, pos = unbc_vclock(b, pos)
    (n,) = _st.unpack_from("<Q", b, pos)
    pos += 8
    entries = {}
    for _ in range(n):
        (k,) = _st.unpack_from("<I", b, pos)
        ec, pos = unbc_vclock(b, pos + 4)
        (m,) = _st.unpack_from("<Q", b, pos)
        pos += 8
        vals = []
        for _ in range(m):
            vc, pos = unbc_vclock(b, pos)
            (v,) = _st.unpack_from("<Q", b, pos)
            pos += 8
            vals.append((vc, v))
        entries[k] = (ec, vals)
    (d,) = _st.unpack_from("<Q", b, pos)
    pos += 8
    deferred = {}
    for _ in range(d):
        rm, pos = unbc_vclock(b, pos)
        (k,) = _st.unpack_from("<Q", b, pos)
        keys = {_st.unpack_from("<I", b, pos + 8 + 4 * i)[0] for i in range(k)}
        pos += 8 + 4 * k
        deferred.setdefault(tuple(sorted(rm.items())), set()).update(keys)
    return clock, entries, deferred, pos


def unbc_vclock(b: bytes, pos: int = 0):
    (n,) = _st.unpack_from("<Q", b, pos)
    pos += 8
    dots = {}
    for _ in range(n):
        a, c = _st.unpack_from("<IQ", b, pos)
        dots[a] = c
        pos += 12
    return dots, pos


def unbc_gset(b: bytes, pos: int = 0):
    (n,) = _st.unpack_from("<Q", b, pos)
    vals = [_st.unpack_from("<Q", b, pos + 8 + 8 * i)[0] for i in range(n)]
    return set(vals), pos + 8 + 8 * n


def unbc_orswot(b: bytes, pos: int = 0):
    """-> (clock, entries {m: dots}, deferred {tuple(sorted rm items): set(members)}, pos); removes
    with the same clock merge their sets, as the HashMap<VClock, HashSet<M>> does."""
    clock, pos = unbc_vclock(b, pos)
    (n,) = _st.unpack_from("<Q", b, pos)
    pos += 8
    entries = {}
    for _ in range(n):
        (m,) = _st.unpack_from("<Q", b, pos)
        entries[m], pos = unbc_vclock(b, pos + 8)
    (d,) = _st.unpack_from("<Q", b, pos)
    pos += 8
    deferred = {}
    for _ in range(d):
        rm, pos = unbc_vclock(b, pos)
        (k,) = _st.unpack_from("<Q", b, pos)
        mem = {_st.unpack_from("<Q", b, pos + 8 + 8 * i)[0] for i in range(k)}
        pos += 8 + 8 * k
        deferred.setdefault(tuple(sorted(rm.items())), set()).update(mem)
    return clock, entries, deferred, pos


def bc_map_obj(m, aid, kid, mid=None, iid=None) -> bytes:
    """A value-typed Map object (Map<u32, GCounter / PNCounter / Orswot<u64>, u32>, map.rs:31-47 with
    gcounter.rs:25-28, pncounter.rs:28-32, orswot.rs:20-25 inside) -> bincode, its dense actor / key /
    member indices mapped to ids through aid / kid / mid (ascending sequences, so index order is id
    order).  Entries by key (BTreeMap), Orswot members ascending (a HashMap: any order decodes the
    same; ascending is what crdt_map_*_egress writes), removes in the dict's order."""
    vc = lambda v: bc_vclock({int(aid[a]): c for a, c in v.dots.items()})  # noqa: E731

    def val(v):
        if isinstance(v, Map):  # the nested Map<u32, MVReg<u64>> (iid maps its keys)
            out = vc(v.clock) + _st.pack("<Q", len(v.entries))
            for j in sorted(v.entries):
                ie = v.entries[j]
                out += _st.pack("<I", int(iid[j])) + vc(ie.clock) + _st.pack("<Q", len(ie.val.vals))
                for c, x in ie.val.vals:
                    out += vc(c) + _st.pack("<Q", int(x))
            out += _st.pack("<Q", len(v.deferred))
            for rm, ks in v.deferred.items():
                kk = sorted(int(iid[x]) for x in ks)
                out += vc(rm) + _st.pack("<Q", len(kk)) + b"".join(_st.pack("<I", x) for x in kk)
            return out
        if isinstance(v, GCounter):
            return vc(v.inner)
        if isinstance(v, PNCounter):
            return vc(v.p.inner) + vc(v.n.inner)
        out = vc(v.clock) + _st.pack("<Q", len(v.entries))
        for x in sorted(v.entries):
            out += _st.pack("<Q", int(mid[x])) + vc(v.entries[x])
        out += _st.pack("<Q", len(v.deferred))
        for rm, mems in v.deferred.items():
            ms = sorted(int(mid[x]) for x in mems)
            out += vc(rm) + _st.pack("<Q", len(ms)) + b"".join(_st.pack("<Q", x) for x in ms)
        return out

    out = vc(m.clock) + _st.pack("<Q", len(m.entries))
    for k in sorted(m.entries):
        e = m.entries[k]
        out += _st.pack("<I", int(kid[k])) + vc(e.clock) + val(e.val)
    out += _st.pack("<Q", len(m.deferred))
    for rm, keys in m.deferred.items():
        kk = sorted(int(kid[x]) for x in keys)
        out += vc(rm) + _st.pack("<Q", len(kk)) + b"".join(_st.pack("<I", x) for x in kk)
    return out


def unbc_map_obj(b: bytes, vnew, aid, kid, mid=None, pos: int = 0, iid=None):
    """Inverse of bc_map_obj -> (Map object over dense indices, pos); vnew = GCounter, PNCounter,
    Orswot or "nested" (Map<K2, MVReg<u64>> values, inner keys through iid).  Removes with equal clocks
    union their sets (the HashMap keyed by the clock)."""
    ai = {int(x): i for i, x in enumerate(aid)}
    ki = {int(x): i for i, x in enumerate(kid)}
    mi = {int(x): i for i, x in enumerate(mid)} if mid is not None else {}
    ii = {int(x): i for i, x in enumerate(iid)} if iid is not None else {}
    nested = vnew == "nested"
    if nested:
        vnew = lambda: Map(MVReg)  # noqa: E731

    def vc(pos):
        d, pos = unbc_vclock(b, pos)
        return VClock({ai[a]: c for a, c in d.items()}), pos

    m = Map(vnew)
    m.clock, pos = vc(pos)
    (n,) = _st.unpack_from("<Q", b, pos)
    pos += 8
    for _ in range(n):
        (k,) = _st.unpack_from("<I", b, pos)
        ec, pos = vc(pos + 4)
        v = vnew()
        if nested:
            v.clock, pos = vc(pos)
            (n2,) = _st.unpack_from("<Q", b, pos)
            pos += 8
            for _ in range(n2):
                (j,) = _st.unpack_from("<I", b, pos)
                iec, pos = vc(pos + 4)
                (nv,) = _st.unpack_from("<Q", b, pos)
                pos += 8
                vals = []
                for _ in range(nv):
                    c, pos = vc(pos)
                    (x,) = _st.unpack_from("<Q", b, pos)
                    pos += 8
                    vals.append((c, x))
                v.entries[ii[j]] = MapEntry(iec, MVReg(vals))
            (nd,) = _st.unpack_from("<Q", b, pos)
            pos += 8
            for _ in range(nd):
                rm, pos = vc(pos)
                (j,) = _st.unpack_from("<Q", b, pos)
                v.deferred.setdefault(rm, set()).update(ii[_st.unpack_from("<I", b, pos + 8 + 4 * i)[0]] for i in range(j))
                pos += 8 + 4 * j
        elif vnew is GCounter:
            v.inner, pos = vc(pos)
        elif vnew is PNCounter:
            v.p.inner, pos = vc(pos)
            v.n.inner, pos = vc(pos)
        else:
            v.clock, pos = vc(pos)
            (ne,) = _st.unpack_from("<Q", b, pos)
            pos += 8
            for _ in range(ne):
                (x,) = _st.unpack_from("<Q", b, pos)
                v.entries[mi[x]], pos = vc(pos + 8)
            (nd,) = _st.unpack_from("<Q", b, pos)
            pos += 8
            for _ in range(nd):
                rm, pos = vc(pos)
                (j,) = _st.unpack_from("<Q", b, pos)
                v.deferred.setdefault(rm, set()).update(mi[_st.unpack_from("<Q", b, pos + 8 + 8 * i)[0]]
                                                        for i in range(j))
                pos += 8 + 8 * j
        m.entries[ki[k]] = MapEntry(ec, v)
    (d,) = _st.unpack_from("<Q", b, pos)
    pos += 8
    for _ in range(d):
        rm, pos = vc(pos)
        (j,) = _st.unpack_from("<Q", b, pos)
        m.deferred.setdefault(rm, set()).update(ki[_st.unpack_from("<I", b, pos + 8 + 4 * i)[0]] for i in range(j))
        pos += 8 + 4 * j
    return m, pos


def frames(blobs, align: int = 4):
    """Concatenate frames (each padded to `align` bytes by construction) -> (bytes, offsets)."""
    off = [0]
    for x in blobs:
        assert len(x) % align == 0
        off.append(off[-1] + len(x))
    return b"".join(blobs), off
