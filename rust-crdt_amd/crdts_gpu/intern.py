"""Ingest / egress between reference-shaped states and the dense SoA layout.

The reference keys clocks by arbitrary `Actor: Ord + Clone + Hash` values (vclock.rs:28-29)
and sets/ORSWOTs by `Member: Clone + Hash + Eq` (orswot.rs:15-16).  The kernels work on dense
indices: an `Index` interns ids to 0..n-1 in first-seen order.  Egress drops zero counters,
matching `apply_dot`, which never stores a 0 (vclock.rs:155-159), so dense -> map -> dense
round-trips exactly.
"""
from __future__ import annotations

from typing import Dict, Hashable, Iterable, List, Mapping, Sequence

import numpy as np


class Index:
    def __init__(self, ids: Iterable[Hashable] = ()):
        self.ids: List[Hashable] = []
        self.pos: Dict[Hashable, int] = {}
        for i in ids:
            self.intern(i)

    def intern(self, x: Hashable) -> int:
        p = self.pos.get(x)
        if p is None:
            p = len(self.ids)
            self.pos[x] = p
            self.ids.append(x)
        return p

    def __len__(self) -> int:
        return len(self.ids)


def clocks_to_dense(clocks: Sequence[Mapping[Hashable, int]], index: Index, width: int = 0) -> np.ndarray:
    """Rows of {actor: counter} maps -> (len, max(width, |index|)) u64 matrix."""
    for c in clocks:
        for a in c:
            index.intern(a)
    W = max(width, len(index))
    out = np.zeros((len(clocks), W), dtype=np.uint64)
    for r, c in enumerate(clocks):
        for a, v in c.items():
            if v < 0 or v >= 2**64:
                raise ValueError(f"counter {v} for actor {a!r} is not a u64")
            out[r, index.pos[a]] = v
    return out


def dense_to_clocks(rows: np.ndarray, index: Index) -> List[Dict[Hashable, int]]:
    rows = np.asarray(rows).view(np.uint64)
    if rows.ndim == 1:
        rows = rows[None, :]
    out = []
    for row in rows:
        nz = np.nonzero(row)[0]
        out.append({index.ids[i]: int(row[i]) for i in nz})
    return out


def sets_to_bitmap(sets: Sequence[Iterable[Hashable]], index: Index, universe: int = 0) -> np.ndarray:
    for s in sets:
        for e in s:
            index.intern(e)
    U = max(universe, len(index))
    words = max(1, (U + 63) // 64)
    out = np.zeros((len(sets), words), dtype=np.uint64)
    for r, s in enumerate(sets):
        for e in s:
            p = index.pos[e]
            out[r, p // 64] |= np.uint64(1) << np.uint64(p % 64)
    return out


def bitmap_to_sets(words: np.ndarray, index: Index) -> List[set]:
    words = np.asarray(words).view(np.uint64)
    if words.ndim == 1:
        words = words[None, :]
    out = []
    for row in words:
        s = set()
        for w, x in enumerate(row.tolist()):
            while x:
                b = (x & -x).bit_length() - 1
                s.add(index.ids[w * 64 + b])
                x &= x - 1
        out.append(s)
    return out
