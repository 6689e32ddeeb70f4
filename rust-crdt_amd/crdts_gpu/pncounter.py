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


def read(states: torch.Tensor) -> list:
    """PNCounter::read (pncounter.rs:110-115): exact P - N per row, on the host."""
    import numpy as np
    a = states.detach().cpu().numpy().view(np.uint64)
    rows = a.reshape(-1, a.shape[-1])
    A = rows.shape[1] // 2
    return [sum(int(x) for x in r[:A]) - sum(int(x) for x in r[A:]) for r in rows]
