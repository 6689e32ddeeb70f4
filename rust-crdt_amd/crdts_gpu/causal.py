"""Batched causal helpers on dense clock rows (reference: src/vclock.rs, src/traits.rs:39-42).

    glb(x, y)            VClock::glb           (vclock.rs:246-259) per row pair: pointwise min
    forget(x, y)         Causal::forget        (vclock.rs:95-105; GCounter gcounter.rs:51-53,
                                                PNCounter pncounter.rs:78-81): keep x iff x > y
    intersection(x, y)   VClock::intersection  (vclock.rs:218-227) per row pair: keep x[a] iff
                                                y[a] == x[a]
    partial_cmp(x, y)    VClock::partial_cmp   (vclock.rs:68-80) per row pair, coded
                         EQUAL 0 / GREATER 1 / LESS -1 / CONCURRENT 2 (None)
    concurrent(x, y)     VClock::concurrent    (vclock.rs:201-203): partial_cmp is None
    cmp_matrix(x)        partial_cmp of every pair of N clocks: (N, N) codes

Rows are (N, A) int64/uint64 device tensors (actor interned to a column, absent = 0) or a single
(A,) row; `out` of glb / forget may be `x` itself (in place, like the reference's &mut self).
"""
from __future__ import annotations

from typing import Optional

import torch

from .context import Context, dptr

EQUAL, GREATER, LESS, CONCURRENT = 0, 1, -1, 2
_GLB, _FORGET, _INTERSECTION = 1, 2, 3


def _rows(t: torch.Tensor, what: str) -> torch.Tensor:
    r = t.unsqueeze(0) if t.dim() == 1 else t
    if r.dim() != 2:
        raise ValueError(f"{what}: expected (N, A) or (A,), got {tuple(t.shape)}")
    if r.shape[1] > 0 and r.stride(1) != 1:
        raise ValueError(f"{what}: rows must be contiguous")
    return r


def _pair_op(op: int, name: str, x: torch.Tensor, y: torch.Tensor, out: Optional[torch.Tensor],
             ctx: Optional[Context]) -> torch.Tensor:
    ctx = ctx or Context.default(x.device.index)
    ctx.check_tensor(x, f"{name}(x)")
    ctx.check_tensor(y, f"{name}(y)")
    x2, y2 = _rows(x, name), _rows(y, name)
    if x2.shape != y2.shape:
        raise ValueError(f"{name}: x {tuple(x.shape)} and y {tuple(y.shape)} differ")
    if out is None:
        out = torch.empty_like(x)
    ctx.check_tensor(out, f"{name}(out)")
    o2 = _rows(out, name)
    if o2.shape != x2.shape:
        raise ValueError(f"{name}: out must be {tuple(x.shape)}")
    N, A = x2.shape
    ctx.call("crdt_vclock_pair_op", op, dptr(o2), dptr(x2), dptr(y2), N, A, o2.stride(0), x2.stride(0),
             y2.stride(0))
    return out


def glb(x: torch.Tensor, y: torch.Tensor, out: Optional[torch.Tensor] = None,
        ctx: Optional[Context] = None) -> torch.Tensor:
    return _pair_op(_GLB, "causal.glb", x, y, out, ctx)


def forget(x: torch.Tensor, y: torch.Tensor, out: Optional[torch.Tensor] = None,
           ctx: Optional[Context] = None) -> torch.Tensor:
    return _pair_op(_FORGET, "causal.forget", x, y, out, ctx)


def intersection(x: torch.Tensor, y: torch.Tensor, out: Optional[torch.Tensor] = None,
                 ctx: Optional[Context] = None) -> torch.Tensor:
    return _pair_op(_INTERSECTION, "causal.intersection", x, y, out, ctx)


def partial_cmp(x: torch.Tensor, y: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    ctx = ctx or Context.default(x.device.index)
    ctx.check_tensor(x, "causal.partial_cmp(x)")
    ctx.check_tensor(y, "causal.partial_cmp(y)")
    x2, y2 = _rows(x, "causal.partial_cmp"), _rows(y, "causal.partial_cmp")
    if x2.shape != y2.shape:
        raise ValueError(f"causal.partial_cmp: x {tuple(x.shape)} and y {tuple(y.shape)} differ")
    N, A = x2.shape
    out = torch.empty(N, dtype=torch.int8, device=x.device)
    ctx.call("crdt_vclock_partial_cmp", dptr(x2), dptr(y2), N, A, x2.stride(0), y2.stride(0), dptr(out))
    return out[0] if x.dim() == 1 else out


def concurrent(x: torch.Tensor, y: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    return partial_cmp(x, y, ctx) == CONCURRENT


def cmp_matrix(x: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    ctx = ctx or Context.default(x.device.index)
    ctx.check_tensor(x, "causal.cmp_matrix(x)")
    x2 = _rows(x, "causal.cmp_matrix")
    N, A = x2.shape
    out = torch.empty((N, N), dtype=torch.int8, device=x.device)
    ctx.call("crdt_vclock_cmp_matrix", dptr(x2), N, A, x2.stride(0), dptr(out))
    return out


def read_sums(kind: str, states: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    """(N, 2) int64 (lo, hi) words of the exact per-row read() (gcounter / pncounter)."""
    ctx = ctx or Context.default(states.device.index)
    ctx.check_tensor(states, f"{kind}.read(states)")
    s2 = _rows(states, f"{kind}.read")
    N, W = s2.shape
    if kind == "pncounter" and W % 2:
        raise ValueError("pncounter.read: rows are P ‖ N, width must be even")
    A = W // 2 if kind == "pncounter" else W
    out = torch.empty((N, 2), dtype=torch.int64, device=states.device)
    ctx.call(f"crdt_{kind}_read", dptr(s2), N, A, s2.stride(0), dptr(out))
    return out


def words_to_ints(words: torch.Tensor, signed: bool) -> list:
    """Egress of (N, 2) (lo, hi) 128-bit words to Python ints (BigUint / BigInt values)."""
    import numpy as np
    w = words.detach().cpu().numpy().view(np.uint64)
    out = []
    for lo, hi in w.reshape(-1, 2).tolist():
        v = (int(hi) << 64) | int(lo)
        if signed and v >= 1 << 127:
            v -= 1 << 128
        out.append(v)
    return out
