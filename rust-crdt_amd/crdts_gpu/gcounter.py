"""Batched `GCounter` merge (reference: src/gcounter.rs:44-48 — VClock merge on `inner`).

Dense layout: (R, A) or (G, R, A) u64 counters, actor interned to a column.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lattice
from .context import Context


def lub_many(states: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
             ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.lub_many("gcounter", ctx, states, out=out, accumulate=accumulate)


def merge_batch(self_states: torch.Tensor, other_states: torch.Tensor,
                ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.merge_batch("gcounter", ctx, self_states, other_states)


def read(states: torch.Tensor, ctx: Optional[Context] = None) -> list:
    """GCounter::read (gcounter.rs:70-72) of every row (N, A) or of one (A,) state: the exact sum,
    as 128-bit words on the device (crdt_gcounter_read), returned as Python ints (BigUint)."""
    from . import causal
    vals = causal.words_to_ints(causal.read_sums("gcounter", states, ctx), signed=False)
    return vals[0] if states.dim() == 1 else vals
