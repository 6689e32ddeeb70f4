"""Batched `GSet` (reference: src/gset.rs).  Elements are interned to bit positions
(`intern.Interner`); a replica row is ceil(U/64) u64 words, bit e set iff element e is in the set.

    lub_many(states)            CvRDT::merge folded (gset.rs:38-40 -> insert :69-71): bitwise OR
    merge_batch(self, other)    (N, W) in place: self[i].merge(other[i])
    apply(states, idx, e, U)    CmRDT::apply = insert (gset.rs:46-48, :69-71), ops in stream order
    contains(states, e)         GSet::contains (gset.rs:83-85) of one element per row
    read(states, elems)         GSet::read (gset.rs:103-105): each row's elements, ascending
    ingest / egress             the serde (bincode 1.x) wire form of GSet<u64> (gset.rs:8-10)

The merges, apply and the wire form are HIP launches through the C ABI (`crdt_gset_*`).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from . import _lattice, apply as _apply, wire as _wire
from .context import Context


def lub_many(states: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
             ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.lub_many("gset", ctx, states, out=out, accumulate=accumulate)


def merge_batch(self_states: torch.Tensor, other_states: torch.Tensor,
                ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.merge_batch("gset", ctx, self_states, other_states)


def apply(states: torch.Tensor, state_idx: torch.Tensor, element: torch.Tensor, universe: int,
          ctx: Optional[Context] = None) -> int:
    """states[state_idx[i]].insert(element[i]) for every op; returns the number of malformed ops
    (state or element out of range), which are skipped."""
    return _apply.apply_inserts(states, state_idx, element, universe, ctx=ctx)


def contains(states: torch.Tensor, element: torch.Tensor) -> torch.Tensor:
    """(N,) bool: row i holds element[i] (an interned bit position; a position past the row is
    not held, as an element never inserted)."""
    if states.dim() != 2 or element.shape != (states.shape[0],):
        raise ValueError(f"gset.contains: states (N, W) and element (N,), got {tuple(states.shape)} / "
                         f"{tuple(element.shape)}")
    e = element.to(device=states.device, dtype=torch.int64)
    inside = (e >= 0) & (e < states.shape[1] * 64)
    w = torch.where(inside, e // 64, torch.zeros_like(e))
    words = states.gather(1, w.unsqueeze(1)).squeeze(1)
    return inside & (((words >> (e % 64)) & 1) != 0)


def read(states: torch.Tensor, elems: Optional[torch.Tensor] = None) -> List[list]:
    """Each row's members in ascending bit order, as element values when `elems` (the interning
    dictionary, position -> value) is given, else as bit positions."""
    rows = states.detach().cpu().contiguous().view(torch.uint8).numpy()
    import numpy as np
    bits = np.unpackbits(rows.reshape(rows.shape[0], -1), axis=1, bitorder="little")
    d = None if elems is None else elems.detach().cpu().tolist()
    out = []
    for r in bits:
        pos = np.flatnonzero(r).tolist()
        out.append(pos if d is None else [d[p] for p in pos])
    return out


ingest = _wire.gset_ingest
egress = _wire.gset_egress
