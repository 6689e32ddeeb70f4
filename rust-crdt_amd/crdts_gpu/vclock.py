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

Each is one HIP launch through the C ABI (`crdt_vclock_*`, include/crdt_gpu.h); this module only
shapes arguments.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lattice, apply as _apply, causal as _causal, wire as _wire
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
