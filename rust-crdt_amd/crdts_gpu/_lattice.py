"""Shared host logic of the max / OR lattice lubs (VClock, GCounter, PNCounter, GSet)."""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch

from . import _abi
from .context import Context, dptr


def _geometry(states: torch.Tensor, what: str):
    if states.dim() == 2:
        R, W = states.shape
        G, gstride = 1, 0
        rstride = states.stride(0)
    elif states.dim() == 3:
        G, R, W = states.shape
        gstride, rstride = states.stride(0), states.stride(1)
    else:
        raise ValueError(f"{what}: expected (R, W) or (G, R, W), got {tuple(states.shape)}")
    if W > 0 and states.stride(-1) != 1:
        raise ValueError(f"{what}: last dimension must be contiguous")
    return G, R, W, rstride, gstride


def lub_many(kind: str, ctx: Optional[Context], states: torch.Tensor, width_div: int = 1,
             out: Optional[torch.Tensor] = None, accumulate: bool = False) -> torch.Tensor:
    ctx = ctx or Context.default(states.device.index)
    ctx.check_tensor(states, f"{kind}.lub_many(states)")
    G, R, W, rstride, gstride = _geometry(states, f"{kind}.lub_many")
    if W % width_div:
        raise ValueError(f"{kind}.lub_many: row width {W} not a multiple of {width_div}")
    shape = (W,) if states.dim() == 2 else (G, W)
    if out is None:
        if accumulate:
            raise ValueError(f"{kind}.lub_many: accumulate=True needs `out`")
        out = torch.empty(shape, dtype=states.dtype, device=states.device)
    ctx.check_tensor(out, f"{kind}.lub_many(out)")
    if tuple(out.shape) != shape or out.stride(-1) != 1:
        raise ValueError(f"{kind}.lub_many: out must be {shape} with a contiguous last dim")
    ostride = out.stride(0) if out.dim() == 2 else W
    ctx.call(f"crdt_{kind}_lub_many", dptr(states), G, R, W // width_div, rstride, gstride,
             dptr(out), ostride, _abi.CRDT_ACCUMULATE if accumulate else 0)
    return out


def merge_batch(kind: str, ctx: Optional[Context], self_states: torch.Tensor,
                other_states: torch.Tensor, width_div: int = 1) -> torch.Tensor:
    ctx = ctx or Context.default(self_states.device.index)
    ctx.check_tensor(self_states, f"{kind}.merge_batch(self)")
    ctx.check_tensor(other_states, f"{kind}.merge_batch(other)")
    if self_states.dim() != 2 or self_states.shape != other_states.shape:
        raise ValueError(f"{kind}.merge_batch: self and other must both be (N, W), got "
                         f"{tuple(self_states.shape)} / {tuple(other_states.shape)}")
    N, W = self_states.shape
    if W % width_div:
        raise ValueError(f"{kind}.merge_batch: row width {W} not a multiple of {width_div}")
    if self_states.stride(1) != 1 or other_states.stride(1) != 1:
        raise ValueError(f"{kind}.merge_batch: rows must be contiguous")
    ctx.call(f"crdt_{kind}_merge_batch", dptr(self_states), dptr(other_states), N, W // width_div,
             self_states.stride(0), other_states.stride(0))
    return self_states


_WDIV = {"vclock": 1, "gcounter": 1, "pncounter": 2, "gset": 1}


def segments(items: Sequence[Tuple[str, torch.Tensor, torch.Tensor]], ctx: Context, accumulate: bool = False):
    """ctypes crdt_lub_segment array for (kind, states (R, W) / (G, R, W), out (W,) / (G, W))."""
    arr = (_abi.LubSegment * max(1, len(items)))()
    for i, (kind, states, out) in enumerate(items):
        if kind not in _WDIV:
            raise ValueError(f"lub_many_multi: unknown kind {kind}")
        ctx.check_tensor(states, f"lub_many_multi[{i}].states")
        ctx.check_tensor(out, f"lub_many_multi[{i}].out")
        G, R, W, rstride, gstride = _geometry(states, f"lub_many_multi[{i}]")
        shape = (W,) if states.dim() == 2 else (G, W)
        if W % _WDIV[kind] or tuple(out.shape) != shape or out.stride(-1) != 1:
            raise ValueError(f"lub_many_multi[{i}]: out must be {shape}, W a multiple of {_WDIV[kind]}")
        sg = arr[i]
        sg.kind, sg.in_, sg.G, sg.R, sg.A = _abi.CRDT_KIND[kind], states.data_ptr(), G, R, W // _WDIV[kind]
        sg.row_stride, sg.group_stride = rstride, gstride
        sg.out, sg.out_stride = out.data_ptr(), (out.stride(0) if out.dim() == 2 else W)
        sg.flags = _abi.CRDT_ACCUMULATE if accumulate else 0
    return arr


def lub_many_multi(items: Sequence[Tuple[str, torch.Tensor, torch.Tensor]], ctx: Optional[Context] = None,
                   accumulate: bool = False) -> List[torch.Tensor]:
    """Several lattice lubs in one launch per join op (crdt_lub_many_multi): items are
    (kind, states, out); each out gets exactly what `<kind>.lub_many(states, out=out)` writes."""
    if not items:
        return []
    ctx = ctx or Context.default(items[0][1].device.index)
    arr = segments(items, ctx, accumulate)
    ctx.call("crdt_lub_many_multi", arr, len(items))
    return [o for _, _, o in items]
