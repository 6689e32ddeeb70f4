"""Batched `PNCounter` merge (reference: src/pncounter.rs:70-75 — P and N merged independently).

Dense layout: a replica row is 2*A u64 words, P counters in [0, A), N counters in [A, 2A),
so one lub over rows of 2A words is the dual max.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lattice
from .context import Context


def pack(p: torch.Tensor, n: torch.Tensor) -> torch.Tensor:
    """Concatenate P and N counter matrices along the actor axis (the dense row layout)."""
    return torch.cat([p, n], dim=-1)


def lub_many(states: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
             ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.lub_many("pncounter", ctx, states, width_div=2, out=out, accumulate=accumulate)


def merge_batch(self_states: torch.Tensor, other_states: torch.Tensor,
                ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.merge_batch("pncounter", ctx, self_states, other_states, width_div=2)


def read(states: torch.Tensor, ctx: Optional[Context] = None) -> list:
    """PNCounter::read (pncounter.rs:110-115) of every row (N, 2A) = P ‖ N or of one (2A,) state:
    exact P - N as 128-bit two's complement on the device (crdt_pncounter_read), returned as
    Python ints (BigInt)."""
    from . import causal
    vals = causal.words_to_ints(causal.read_sums("pncounter", states, ctx), signed=True)
    return vals[0] if states.dim() == 1 else vals
