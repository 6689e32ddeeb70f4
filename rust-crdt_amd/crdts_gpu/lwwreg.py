"""Batched `LWWReg<u64 val, u64 marker>` merge (reference: src/lwwreg.rs:43-45 -> update :84-98).

`FunkyCvRDT::merge` returns `Err(ConflictingMarker)` when the markers are equal and the values
differ, leaving the register unchanged.  Batched forms:

    lub_many(marker, val)   (R,) or (G, R) -> LwwLub(marker (G,), val (G,), first_conflict (G,))
        the fold acc = r[0]; for r in r[1..]: acc.merge(r) with every Err leaving acc unchanged;
        first_conflict[g] = index of the first merge returning Err, or -1 (u64::MAX) if none.
    merge_batch(self_m, self_v, other_m, other_v) -> conflict (N,) uint8, in place on self.
"""
from __future__ import annotations

from typing import NamedTuple, Optional

import torch

from . import _abi
from .context import Context, dptr

NO_CONFLICT = -1  # u64::MAX bit pattern in an int64 tensor


class LwwLub(NamedTuple):
    marker: torch.Tensor
    val: torch.Tensor
    first_conflict: torch.Tensor


def lub_many(marker: torch.Tensor, val: torch.Tensor, ctx: Optional[Context] = None,
             init: Optional[tuple] = None) -> LwwLub:
    """`init=(marker, val)` continues the fold from that state (CRDT_ACCUMULATE): every replica
    is then merged into it and first_conflict indexes this call's replicas."""
    ctx = ctx or Context.default(marker.device.index)
    ctx.check_tensor(marker, "lwwreg.lub_many(marker)")
    ctx.check_tensor(val, "lwwreg.lub_many(val)")
    if marker.shape != val.shape or marker.dim() not in (1, 2):
        raise ValueError("lwwreg.lub_many: marker and val must share a (R,) or (G, R) shape")
    squeeze = marker.dim() == 1
    m2 = marker.reshape(1, -1) if squeeze else marker
    v2 = val.reshape(1, -1) if squeeze else val
    if m2.stride(1) != 1 or v2.stride(1) != 1 or m2.stride(0) != v2.stride(0):
        raise ValueError("lwwreg.lub_many: rows must be contiguous with equal strides")
    G, R = m2.shape
    flags = 0
    if init is not None:
        om = init[0].reshape(G).to(marker.dtype).clone()
        ov = init[1].reshape(G).to(marker.dtype).clone()
        flags = _abi.CRDT_ACCUMULATE
    else:
        om = torch.empty(G, dtype=marker.dtype, device=marker.device)
        ov = torch.empty_like(om)
    fc = torch.empty_like(om)
    ctx.call("crdt_lwwreg_lub_many", dptr(m2), dptr(v2), G, R, m2.stride(0) if G > 1 else R,
             dptr(om), dptr(ov), dptr(fc), flags)
    if squeeze:
        return LwwLub(om[0], ov[0], fc[0])
    return LwwLub(om, ov, fc)


def merge_batch(self_marker: torch.Tensor, self_val: torch.Tensor, other_marker: torch.Tensor,
                other_val: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    ctx = ctx or Context.default(self_marker.device.index)
    ts = (self_marker, self_val, other_marker, other_val)
    for i, t in enumerate(ts):
        ctx.check_tensor(t, f"lwwreg.merge_batch(arg{i})")
        if t.dim() != 1 or not t.is_contiguous() or t.shape != self_marker.shape:
            raise ValueError("lwwreg.merge_batch: four contiguous (N,) tensors expected")
    N = self_marker.shape[0]
    conflict = torch.empty(N, dtype=torch.uint8, device=self_marker.device)
    ctx.call("crdt_lwwreg_merge_batch", *(dptr(t) for t in ts), N, dptr(conflict))
    return conflict
