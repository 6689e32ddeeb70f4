"""Batched `CmRDT::apply` of op streams to many dense states (reference: vclock.rs:125-127 /
:155-159, gcounter.rs:39-41, pncounter.rs:62-67, gset.rs:46-48).

    apply_dots(kind, states, state_idx, actor, counter[, dir])   kind: vclock / gcounter / pncounter
    apply_inserts(states, state_idx, element)                     GSet

states (N, W) device rows, updated in place; ops as device tensors (state_idx / actor / element
int32, counter int64 holding u64 bits, dir uint8: 0 = Dir::Pos, 1 = Dir::Neg).  The ops commute
(per-cell max / set-bit), so the result equals applying them one by one in any order.  Returns
the number of out-of-range ops that were skipped (0 for a valid batch)."""
from __future__ import annotations

from typing import Optional

import torch

from .context import Context, dptr


def _ops(ctx, t, dtypes, what, n):
    if t.device.type != "cuda" or t.device.index != ctx.device:
        raise ValueError(f"{what}: expected a cuda:{ctx.device} tensor")
    if t.dtype not in dtypes or not t.is_contiguous() or t.dim() != 1 or t.shape[0] != n:
        raise ValueError(f"{what}: expected a contiguous ({n},) tensor of {dtypes}")


def _states(ctx, states, what):
    ctx.check_tensor(states, what)
    if states.dim() != 2 or (states.shape[1] > 0 and states.stride(1) != 1):
        raise ValueError(f"{what}: states must be (N, W) with contiguous rows")


def apply_dots(kind: str, states: torch.Tensor, state_idx: torch.Tensor, actor: torch.Tensor,
               counter: torch.Tensor, dir: Optional[torch.Tensor] = None,
               ctx: Optional[Context] = None) -> int:
    ctx = ctx or Context.default(states.device.index)
    _states(ctx, states, f"{kind}.apply")
    n = state_idx.shape[0]
    i32 = (torch.int32, torch.uint32)
    _ops(ctx, state_idx, i32, f"{kind}.apply(state_idx)", n)
    _ops(ctx, actor, i32, f"{kind}.apply(actor)", n)
    _ops(ctx, counter, (torch.int64, torch.uint64), f"{kind}.apply(counter)", n)
    N, W = states.shape
    bad = torch.zeros(1, dtype=torch.int32, device=states.device)
    if kind == "pncounter":
        if dir is None:
            raise ValueError("pncounter.apply: dir required")
        _ops(ctx, dir, (torch.uint8, torch.int8, torch.bool), "pncounter.apply(dir)", n)
        if W % 2:
            raise ValueError("pncounter.apply: rows are P ‖ N, width must be even")
        ctx.call("crdt_pncounter_apply_batch", dptr(states), N, W // 2, states.stride(0), dptr(state_idx),
                 dptr(actor), dptr(counter), dptr(dir), n, dptr(bad))
    elif kind in ("vclock", "gcounter"):
        ctx.call(f"crdt_{kind}_apply_batch", dptr(states), N, W, states.stride(0), dptr(state_idx), dptr(actor),
                 dptr(counter), n, dptr(bad))
    else:
        raise ValueError(f"apply_dots: unknown kind {kind}")
    return int(bad.item())


def apply_inserts(states: torch.Tensor, state_idx: torch.Tensor, element: torch.Tensor, universe: int,
                  ctx: Optional[Context] = None) -> int:
    ctx = ctx or Context.default(states.device.index)
    _states(ctx, states, "gset.apply")
    n = state_idx.shape[0]
    i32 = (torch.int32, torch.uint32)
    _ops(ctx, state_idx, i32, "gset.apply(state_idx)", n)
    _ops(ctx, element, i32, "gset.apply(element)", n)
    N, W = states.shape
    if W * 64 < universe:
        raise ValueError(f"gset.apply: {W} words cannot hold a universe of {universe}")
    bad = torch.zeros(1, dtype=torch.int32, device=states.device)
    ctx.call("crdt_gset_apply_batch", dptr(states), N, universe, states.stride(0), dptr(state_idx), dptr(element),
             n, dptr(bad))
    return int(bad.item())
