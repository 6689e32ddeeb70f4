"""Batched `MVReg<u64, A>` on its own (reference: src/mvreg.rs:112-166; include/crdt_gpu.h "MVReg").

Dense register (the value layout of the Map entry points): slots in Vec order,
    vclk (..., V, A)  value clocks (empty slot <=> all-zero row)
    vval (..., V)     values, u64 ids interned by the caller (merge / apply never compare values)

    lub_many(vclk (G, R, V, A) or (R, V, A), vval)  acc = MVReg::new(); for r: acc.merge(r)  (mvreg.rs:112-128)
    merge_batch(self (N, V, A), other)               self[i].merge(other[i]), in place
    apply_batch(vclk (N, V, A), vval, ops)           reg[i].apply(op) for its ops in order   (mvreg.rs:130-166)
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple, Optional, Sequence

import numpy as np
import torch

from . import _abi
from .context import Context


class MVRegLub(NamedTuple):
    vclk: torch.Tensor   # (G, Vout, A)
    vval: torch.Tensor   # (G, Vout)
    nval: torch.Tensor   # (G,) int32
    flags: torch.Tensor  # (G,) int32


class MVRegCapacityError(RuntimeError):
    """A register holds more values than the output (or its own) slots."""


def _check_regs(ctx, vclk, vval, what, lead):
    ctx.check_tensor(vclk, f"{what}(vclk)")
    ctx.check_tensor(vval, f"{what}(vval)")
    if vclk.dim() != lead + 2 or vval.dim() != lead + 1 or tuple(vclk.shape[:-1]) != tuple(vval.shape):
        raise ValueError(f"{what}: vclk (..., V, A) and vval (..., V) expected")
    V, A = vclk.shape[-2], vclk.shape[-1]
    if vclk.stride(-1) != 1 or vclk.stride(-2) != A or vval.stride(-1) != 1:
        raise ValueError(f"{what}: each register's slots must be packed")
    return V, A


def lub_many(vclk: torch.Tensor, vval: torch.Tensor, vout: int = 4, ctx: Optional[Context] = None,
             check: bool = True, vstate: int = 0) -> MVRegLub:
    """Left fold of each group's replicas from MVReg::new().  A group needing more than `vout`
    values raises MVRegCapacityError (check=True); a fold state overflow reruns with 16 slots."""
    ctx = ctx or Context.default(vclk.device.index)
    squeeze = vclk.dim() == 3
    vc = vclk.unsqueeze(0) if squeeze else vclk
    vv = vval.unsqueeze(0) if squeeze else vval
    V, A = _check_regs(ctx, vc, vv, "mvreg.lub_many", 2)
    G, R = vc.shape[0], vc.shape[1]
    dev = vclk.device
    out_c = torch.empty((G, vout, A), dtype=torch.int64, device=dev)
    out_v = torch.empty((G, vout), dtype=torch.int64, device=dev)
    nval = torch.empty(G, dtype=torch.int32, device=dev)
    flags = torch.empty(G, dtype=torch.int32, device=dev)
    b = _abi.MVRegBatch(G, R, A, V, vc.data_ptr(), vc.stride(1), vc.stride(0), vv.data_ptr(), vv.stride(1),
                        vv.stride(0))
    o = _abi.MVRegOut(vout, vstate, out_c.data_ptr(), out_v.data_ptr(), nval.data_ptr(), flags.data_ptr())
    ctx.call("crdt_mvreg_lub_many", ctypes.byref(b), ctypes.byref(o))
    if check:
        f = int(np.bitwise_or.reduce(flags.cpu().numpy())) if G else 0
        if f & 4 and vstate < 16:
            return lub_many(vclk, vval, vout, ctx, check, vstate=16)
        if f & 4:
            raise MVRegCapacityError("mvreg.lub_many: a register held more than 16 values during the fold")
        if f & 1:
            raise MVRegCapacityError(f"mvreg.lub_many: a register folds to more than vout={vout} values")
    if squeeze:
        return MVRegLub(out_c[0], out_v[0], nval, flags)
    return MVRegLub(out_c, out_v, nval, flags)


def _states(ctx, vclk, vval, what):
    V, A = _check_regs(ctx, vclk, vval, what, 1)
    return _abi.MVRegStates(vclk.shape[0], A, V, vclk.data_ptr(), vclk.stride(0), vval.data_ptr(), vval.stride(0))


def merge_batch(self_vclk: torch.Tensor, self_vval: torch.Tensor, other_vclk: torch.Tensor,
                other_vval: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    """self[i].merge(other[i]) in place on (N, V, A) / (N, V); returns status (N,) int32 (bit 4 =
    more than self's V values: that register is incomplete)."""
    ctx = ctx or Context.default(self_vclk.device.index)
    a = _states(ctx, self_vclk, self_vval, "mvreg.merge_batch(self)")
    b = _states(ctx, other_vclk, other_vval, "mvreg.merge_batch(other)")
    status = torch.empty(a.N, dtype=torch.int32, device=self_vclk.device)
    ctx.call("crdt_mvreg_merge_batch", ctypes.byref(a), ctypes.byref(b), status.data_ptr())
    return status


class MVRegOpBatch(NamedTuple):
    op_off: torch.Tensor    # (N+1,) int64
    clk_row: torch.Tensor   # (n_ops,) int32
    clk_pool: torch.Tensor  # (n_clk, A) int64
    val: torch.Tensor       # (n_ops,) int64


def encode_ops(streams: Sequence, A: int, device) -> MVRegOpBatch:
    """Per-register streams of Op::Put (mvreg.rs:38-47) as (clock, val): clock a mapping actor ->
    counter or a dense row of A counters, val a u64 id."""
    op_off, clk_row, val, pool = [0], [], [], []
    for ops in streams:
        for clock, v in ops:
            r = np.zeros(A, np.uint64)
            if hasattr(clock, "items"):
                for a, c in clock.items():
                    r[int(a)] = np.uint64(c)
            else:
                r[:] = np.asarray(clock, np.uint64)
            clk_row.append(len(pool))
            pool.append(r)
            val.append(int(v))
        op_off.append(len(val))
    pool.append(np.zeros(A, np.uint64))
    t = lambda x, dt: torch.from_numpy(np.asarray(x, dtype=dt)).to(device)  # noqa: E731
    return MVRegOpBatch(t(op_off, np.int64), t(clk_row or [0], np.int32)[:len(clk_row)],
                        torch.from_numpy(np.stack(pool).view(np.int64)).to(device),
                        torch.from_numpy(np.array(val or [0], np.uint64).view(np.int64)).to(device)[:len(val)])


def apply_batch(vclk: torch.Tensor, vval: torch.Tensor, ops: MVRegOpBatch, ctx: Optional[Context] = None) -> torch.Tensor:
    """Apply every register's op stream in place; returns status (N,) int32 (include/crdt_gpu.h)."""
    ctx = ctx or Context.default(vclk.device.index)
    st = _states(ctx, vclk, vval, "mvreg.apply_batch")
    n = ops.val.shape[0]
    if ops.op_off.shape[0] != st.N + 1 or ops.clk_row.shape[0] != n or ops.clk_pool.shape[1] != st.A:
        raise ValueError("mvreg.apply_batch: op_off (N+1,), clk_row (n_ops,), clk_pool (n, A)")
    o = _abi.MVRegOps(n, ops.op_off.data_ptr(), ops.clk_row.data_ptr(), ops.clk_pool.data_ptr(),
                      ops.clk_pool.shape[0], ops.val.data_ptr())
    status = torch.empty(st.N, dtype=torch.int32, device=vclk.device)
    ctx.call("crdt_mvreg_apply_batch", ctypes.byref(st), ctypes.byref(o), status.data_ptr())
    return status
