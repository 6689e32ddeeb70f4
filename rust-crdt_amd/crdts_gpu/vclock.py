"""Batched `VClock` merge (reference: src/vclock.rs).

`CvRDT::merge` for VClock (vclock.rs:130-136) applies every dot of `other` through
`apply_dot` (vclock.rs:155-159): keep the larger counter per actor.  On the dense layout
(actor interned to a column, absent = 0) a fold over replicas is an elementwise max.

    lub_many(states)          states (R, A) -> (A,)   or (G, R, A) -> (G, A)
                              == acc = VClock::new(); for r in replicas { acc.merge(r) }
    merge_batch(self, other)  (N, A) in place: self[i].merge(other[i])
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lattice
from .context import Context


def lub_many(states: torch.Tensor, out: Optional[torch.Tensor] = None, accumulate: bool = False,
             ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.lub_many("vclock", ctx, states, out=out, accumulate=accumulate)


def merge_batch(self_states: torch.Tensor, other_states: torch.Tensor,
                ctx: Optional[Context] = None) -> torch.Tensor:
    return _lattice.merge_batch("vclock", ctx, self_states, other_states)
