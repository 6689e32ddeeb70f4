"""Batched `Orswot<member, actor>` merge (reference: src/orswot.rs:81-149).

Dense layout (members and actors interned to indices):
    clock   (R, A)    or (G, R, A)      replica clocks
    entries (R, M, A) or (G, R, M, A)   per-member dot clocks; member absent <=> row all 0
    deferred removes pooled per group as CSR:
        def_off     host sequence of G+1 offsets (group g owns [def_off[g], def_off[g+1]))
        def_clock   (D, A)   rm clocks
        def_members (D, ceil(M/64)) member bitmaps

lub_many folds each group from Orswot::new() (test/orswot.rs:50-53) and returns
OrswotLub(clock (G, A), entries (G, M, A), def_keep (D,) uint8, def_members (D, Mw)):
def_keep[d] = 1 marks the representative of each surviving deferred remove (first of its
group with that exact rm clock); def_members[d] is then the union of the member sets of all
survivors sharing that clock (orswot.rs:240-249).
"""
from __future__ import annotations

from typing import NamedTuple, Optional, Sequence

import ctypes

import numpy as np
import torch

from . import _abi
from .context import Context, dptr


class OrswotLub(NamedTuple):
    clock: torch.Tensor
    entries: torch.Tensor
    def_keep: Optional[torch.Tensor]
    def_members: Optional[torch.Tensor]


def lub_many(clock: torch.Tensor, entries: torch.Tensor, def_off: Optional[Sequence[int]] = None,
             def_clock: Optional[torch.Tensor] = None, def_members: Optional[torch.Tensor] = None,
             ctx: Optional[Context] = None) -> OrswotLub:
    ctx = ctx or Context.default(clock.device.index)
    ctx.check_tensor(clock, "orswot.lub_many(clock)")
    ctx.check_tensor(entries, "orswot.lub_many(entries)")
    squeeze = clock.dim() == 2
    c = clock.unsqueeze(0) if squeeze else clock
    e = entries.unsqueeze(0) if squeeze else entries
    if c.dim() != 3 or e.dim() != 4:
        raise ValueError("orswot.lub_many: clock (G,R,A) / entries (G,R,M,A) expected")
    G, R, A = c.shape
    if e.shape[0] != G or e.shape[1] != R or e.shape[3] != A:
        raise ValueError(f"orswot.lub_many: entries {tuple(e.shape)} do not match clock {tuple(c.shape)}")
    if c.stride(2) != 1 or e.stride(3) != 1:
        raise ValueError("orswot.lub_many: actor axis must be contiguous")
    M = e.shape[2]
    Mw = (M + 63) // 64
    out_clock = torch.empty((G, A), dtype=clock.dtype, device=clock.device)
    out_entries = torch.empty((G, M, A), dtype=clock.dtype, device=clock.device)
    b = _abi.OrswotBatch()
    b.G, b.R, b.M, b.A = G, R, M, A
    b.clock, b.clock_rstride, b.clock_gstride = c.data_ptr(), c.stride(1), c.stride(0)
    b.entries = e.data_ptr()
    b.entry_mstride, b.entry_rstride, b.entry_gstride = e.stride(2), e.stride(1), e.stride(0)
    o = _abi.OrswotOut()
    o.clock, o.entries = out_clock.data_ptr(), out_entries.data_ptr()
    keep = members_out = None
    off_arr = None
    if def_off is not None:
        off = np.asarray(def_off, dtype=np.uint64)
        if off.shape != (G + 1,):
            raise ValueError(f"orswot.lub_many: def_off must have G+1 = {G + 1} entries")
        D = int(off[-1])
        if D > 0:
            for t, nm in ((def_clock, "def_clock"), (def_members, "def_members")):
                if t is None:
                    raise ValueError(f"orswot.lub_many: {nm} required with deferred removes")
                ctx.check_tensor(t, f"orswot.lub_many({nm})")
                if not t.is_contiguous():
                    raise ValueError(f"orswot.lub_many: {nm} must be contiguous")
            if tuple(def_clock.shape) != (D, A) or tuple(def_members.shape) != (D, Mw):
                raise ValueError(f"orswot.lub_many: def_clock {tuple(def_clock.shape)} / def_members "
                                 f"{tuple(def_members.shape)}; expected ({D},{A}) / ({D},{Mw})")
            off_arr = (ctypes.c_size_t * (G + 1))(*[int(x) for x in off])
            b.def_off = ctypes.cast(off_arr, ctypes.POINTER(ctypes.c_size_t))
            b.def_clock, b.def_members = def_clock.data_ptr(), def_members.data_ptr()
            keep = torch.empty(D, dtype=torch.uint8, device=clock.device)
            members_out = torch.empty((D, Mw), dtype=clock.dtype, device=clock.device)
            o.def_keep, o.def_members = keep.data_ptr(), members_out.data_ptr()
    ctx.call("crdt_orswot_lub_many", ctypes.byref(b), ctypes.byref(o))
    if squeeze:
        return OrswotLub(out_clock[0], out_entries[0], keep, members_out)
    return OrswotLub(out_clock, out_entries, keep, members_out)


def deferred_set(def_clock: torch.Tensor, def_keep: torch.Tensor, def_members: torch.Tensor,
                 lo: int = 0, hi: Optional[int] = None) -> set:
    """Egress of the surviving deferred removes of pool range [lo, hi) to the reference shape
    {(rm clock as a tuple of dense counters, frozenset of member indices)}."""
    keep = def_keep.cpu().numpy()
    clocks = def_clock.cpu().numpy().view(np.uint64)
    mem = def_members.cpu().numpy().view(np.uint64)
    hi = keep.shape[0] if hi is None else hi
    out = set()
    for d in range(lo, hi):
        if keep[d]:
            ms = []
            for w, x in enumerate(mem[d].tolist()):
                while x:
                    bit = (x & -x).bit_length() - 1
                    ms.append(w * 64 + bit)
                    x &= x - 1
            out.add((tuple(int(v) for v in clocks[d]), frozenset(ms)))
    return out
