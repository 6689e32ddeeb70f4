"""Batched `GSet` merge (reference: src/gset.rs:38-40 -> insert :69-71: set union).

Elements are interned to bit positions; a replica row is ceil(U/64) u64 words and the union
of replicas is a bitwise OR.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lattice
from .context import Context


def lub_many(states: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
             ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.lub_many("gset", ctx, states, out=out, accumulate=accumulate)


def merge_batch(self_states: torch.Tensor, other_states: torch.Tensor,
                ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.merge_batch("gset", ctx, self_states, other_states)
