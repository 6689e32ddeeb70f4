"""Batched `VClock` (reference: src/vclock.rs) on dense rows: actor interned to a column, an
absent actor is 0.  Every entry point of the crate's VClock that acts on a batch of clocks:

    lub_many(states)            CvRDT::merge folded (vclock.rs:130-136 -> apply_dot :155-159):
                                states (R, A) -> (A,) or (G, R, A) -> (G, A)
                                == acc = VClock::new(); for r in replicas { acc.merge(r) }
    merge_batch(self, other)    (N, A) in place: self[i].merge(other[i])
    apply(states, idx, a, c)    CmRDT::apply of Dot ops in stream order (vclock.rs:125-127)
    forget / clone_without      Causal::forget (vclock.rs:95-105) / clone_without (:148-152)
    glb                         VClock::glb (vclock.rs:246-259)
    intersection                VClock::intersection (vclock.rs:218-227)
    partial_cmp / concurrent    PartialOrd (vclock.rs:68-80) / concurrent (:201-203), coded
                                causal.EQUAL / GREATER / LESS / CONCURRENT
    cmp_matrix                  partial_cmp of every pair of N clocks
    ingest / egress             the serde (bincode 1.x) wire form (vclock.rs:57-60)
    from_clocks / to_clocks     reference-shaped clocks ({actor: counter} maps, any hashable actor)
                                <-> dense rows, with the actor index kept across calls
    get / inc / is_empty        VClock::get (:207-209), inc (:183-189, the next Dot, the state
                                unchanged) and is_empty (:212-214) for a batch

The ops above are one HIP launch each through the C ABI (`crdt_vclock_*`, include/crdt_gpu.h); the
last two groups are the host-side helpers a caller of the crate's VClock API needs around them.
"""
from __future__ import annotations

from typing import Dict, Hashable, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lattice, apply as _apply, causal as _causal, wire as _wire
from .intern import Index, clocks_to_dense, dense_to_clocks
from .causal import CONCURRENT, EQUAL, GREATER, LESS  # noqa: F401
from .context import Context


def lub_many(states: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
             ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.lub_many("vclock", ctx, states, out=out, accumulate=accumulate)


def merge_batch(self_states: torch.Tensor, other_states: torch.Tensor,
                ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.merge_batch("vclock", ctx, self_states, other_states)


def apply(states: torch.Tensor, state_idx: torch.Tensor, actor: torch.Tensor, counter: torch.Tensor,
          ctx: Optional[Context] = None) -> int:
    """states[state_idx[i]].apply(Dot(actor[i], counter[i])) for i in order; returns the number of
    ops rejected as malformed (state or actor out of range)."""
    return _apply.apply_dots("vclock", states, state_idx, actor, counter, ctx=ctx)


def forget(x: torch.Tensor, y: torch.Tensor, out: Optional[torch.Tensor] = None,
           ctx: Optional[Context] = None) -> torch.Tensor:
    return _causal.forget(x, y, out=out, ctx=ctx)


def clone_without(x: torch.Tensor, base: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    """A new batch: x[i] with every actor whose counter base[i] reaches forgotten."""
    return _causal.forget(x, base, ctx=ctx)


def glb(x: torch.Tensor, y: torch.Tensor, out: Optional[torch.Tensor] = None,
        ctx: Optional[Context] = None) -> torch.Tensor:
    return _causal.glb(x, y, out=out, ctx=ctx)


def intersection(left: torch.Tensor, right: torch.Tensor, out: Optional[torch.Tensor] = None,
                 ctx: Optional[Context] = None) -> torch.Tensor:
    return _causal.intersection(left, right, out=out, ctx=ctx)


def partial_cmp(x: torch.Tensor, y: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    return _causal.partial_cmp(x, y, ctx=ctx)


def concurrent(x: torch.Tensor, y: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    return _causal.concurrent(x, y, ctx=ctx)


def cmp_matrix(x: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    return _causal.cmp_matrix(x, ctx=ctx)


ingest = _wire.vclock_ingest
egress = _wire.vclock_egress


# ---- reference-shaped clocks <-> dense rows, and the per-clock accessors ----------------------------
def from_clocks(clocks: Sequence[Mapping[Hashable, int]], actors: Optional[Index] = None, width: int = 0,
                device=None) -> Tuple[torch.Tensor, Index]:
    """A batch of reference clocks ({actor: counter}, u64 counters) as (N, max(width, |actors|)) int64
    rows (u64 bits) on `device`, actors interned into `actors` (a new Index when None; pass the same
    one to keep columns stable across batches).  Returns (rows, actors)."""
    actors = actors if actors is not None else Index()
    rows = clocks_to_dense(clocks, actors, width)
    t = torch.from_numpy(rows.view(np.int64))
    return (t.to(device) if device is not None else t), actors


def to_clocks(rows: torch.Tensor, actors: Index) -> List[Dict[Hashable, int]]:
    """Dense rows back to reference clocks: zero counters are dropped, as apply_dot never stores one
    (vclock.rs:155-159), so from_clocks / to_clocks round-trip exactly."""
    return dense_to_clocks(rows.detach().cpu().numpy().view(np.uint64), actors)


def _cols(rows: torch.Tensor, actor) -> torch.Tensor:
    if rows.dim() != 2:
        raise ValueError("vclock: rows (N, A) expected")
    a = torch.as_tensor(actor, dtype=torch.int64, device=rows.device)
    if a.dim() == 0:
        a = a.expand(rows.shape[0])
    if a.shape != (rows.shape[0],):
        raise ValueError("vclock: one actor column for all rows, or one per row")
    if bool(((a < 0) | (a >= rows.shape[1])).any()):
        raise ValueError("vclock: actor column out of range")
    return a


def get(rows: torch.Tensor, actor) -> torch.Tensor:
    """VClock::get (vclock.rs:207-209) of every row: the counter of `actor` (a column index, or one per
    row), 0 for an actor the clock does not hold.  (N,) int64 (u64 bits)."""
    a = _cols(rows, actor)
    return rows.gather(1, a[:, None])[:, 0]


def inc(rows: torch.Tensor, actor) -> Tuple[torch.Tensor, torch.Tensor]:
    """VClock::inc (vclock.rs:183-189) of every row: the Dot {actor, get(actor) + 1}; the rows are not
    changed (apply the dots with `apply`).  Returns (actor columns, counters).  A counter at u64::MAX
    raises (the reference's `+ 1` would overflow)."""
    a = _cols(rows, actor)
    c = rows.gather(1, a[:, None])[:, 0]
    if bool((c == -1).any()):
        raise OverflowError("vclock.inc: counter at u64::MAX")
    return a, c + 1


def is_empty(rows: torch.Tensor) -> torch.Tensor:
    """VClock::is_empty (vclock.rs:212-214) of every row: no actor with a nonzero counter.  (N,) bool."""
    if rows.dim() != 2:
        raise ValueError("vclock: rows (N, A) expected")
    return ~(rows != 0).any(1)
