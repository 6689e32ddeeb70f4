"""Batched `Orswot<member, actor>` merge (reference: src/orswot.rs:81-149).

Dense layout (members and actors interned to indices):
    clock   (R, A)    or (G, R, A)      replica clocks
    entries (R, M, A) or (G, R, M, A)   per-member dot clocks; member absent <=> row all 0
    deferred removes pooled per group as CSR:
        def_off     host sequence of G+1 offsets (group g owns [def_off[g], def_off[g+1])), or a
                    (G+1,) int64 device tensor (crdt_orswot_lub_many_doff: no host sync)
        def_clock   (D, A)   rm clocks
        def_members (D, ceil(M/64)) member bitmaps

lub_many folds each group from Orswot::new() (test/orswot.rs:50-53) and returns
OrswotLub(clock (G, A), entries (G, M, A), def_keep (D,) uint8, def_members (D, Mw)):
def_keep[d] = 1 marks the representative of each surviving deferred remove (first of its
group with that exact rm clock); def_members[d] is then the union of the member sets of all
survivors sharing that clock (orswot.rs:240-249).
"""
from __future__ import annotations

from typing import NamedTuple, Optional

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


def lub_many(clock: torch.Tensor, entries: torch.Tensor, def_off=None,
             def_clock: Optional[torch.Tensor] = None, def_members: Optional[torch.Tensor] = None,
             ctx: Optional[Context] = None, def_status: Optional[torch.Tensor] = None) -> OrswotLub:
    """def_off a device tensor: D = def_clock.shape[0] (no host read of the offsets); the offsets are
    checked on the device into `def_status` ((1,) int32 device tensor, bit 0 = invalid offsets) when
    one is given, else checked here (one sync) and a ValueError raised."""
    ctx = ctx or Context.default(clock.device.index)
    if isinstance(def_off, torch.Tensor) and def_off.device.type == "cuda":
        return _lub_many_doff(ctx, clock, entries, def_off, def_clock, def_members, def_status)
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


def _lub_many_doff(ctx, clock, entries, def_off, def_clock, def_members, def_status) -> OrswotLub:
    squeeze = clock.dim() == 2
    c = clock.unsqueeze(0) if squeeze else clock
    e = entries.unsqueeze(0) if squeeze else entries
    ctx.check_tensor(c, "orswot.lub_many(clock)")
    ctx.check_tensor(e, "orswot.lub_many(entries)")
    if c.dim() != 3 or e.dim() != 4 or c.stride(2) != 1 or e.stride(3) != 1:
        raise ValueError("orswot.lub_many: clock (G,R,A) / entries (G,R,M,A) with the actor axis contiguous")
    G, R, A = c.shape
    M = e.shape[2]
    if e.shape[0] != G or e.shape[1] != R or e.shape[3] != A:
        raise ValueError(f"orswot.lub_many: entries {tuple(e.shape)} do not match clock {tuple(c.shape)}")
    Mw = (M + 63) // 64
    if (def_off.dtype not in (torch.int64, torch.uint64) or tuple(def_off.shape) != (G + 1,)
            or not def_off.is_contiguous() or def_off.device.index != ctx.device):
        raise ValueError(f"orswot.lub_many: a device def_off must be a contiguous ({G + 1},) int64 cuda:{ctx.device} tensor")
    D = 0 if def_clock is None else int(def_clock.shape[0])
    b = _abi.OrswotBatch()
    b.G, b.R, b.M, b.A = G, R, M, A
    b.clock, b.clock_rstride, b.clock_gstride = c.data_ptr(), c.stride(1), c.stride(0)
    b.entries = e.data_ptr()
    b.entry_mstride, b.entry_rstride, b.entry_gstride = e.stride(2), e.stride(1), e.stride(0)
    out_clock = torch.empty((G, A), dtype=clock.dtype, device=clock.device)
    out_entries = torch.empty((G, M, A), dtype=clock.dtype, device=clock.device)
    o = _abi.OrswotOut()
    o.clock, o.entries = out_clock.data_ptr(), out_entries.data_ptr()
    keep = members_out = None
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
        b.def_clock, b.def_members = def_clock.data_ptr(), def_members.data_ptr()
        keep = torch.empty(D, dtype=torch.uint8, device=clock.device)
        members_out = torch.empty((D, Mw), dtype=clock.dtype, device=clock.device)
        o.def_keep, o.def_members = keep.data_ptr(), members_out.data_ptr()
    st = def_status
    if st is None:
        st = torch.zeros(1, dtype=torch.int32, device=clock.device)
    elif st.dtype not in (torch.int32, torch.uint32) or st.numel() < 1 or st.device != clock.device:
        raise ValueError("orswot.lub_many: def_status must be an int32 device tensor of >= 1 element")
    ctx.call("crdt_orswot_lub_many_doff", ctypes.byref(b), def_off.data_ptr(), D, ctypes.byref(o), st.data_ptr())
    if def_status is None and int(st.item()) & 1:
        raise ValueError("orswot.lub_many: def_off invalid (def_off[0] != 0, decreasing, or def_off[G] != "
                         "def_clock.shape[0])")
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


# ---------------------------------------------------------------------------------------------
# Batched CmRDT::apply (orswot.rs:55-79, apply_rm :230-250, apply_deferred :281-286)
# ---------------------------------------------------------------------------------------------
class OrswotOpBatch(NamedTuple):
    """Device op streams (crdt_orswot_ops): state s applies ops [op_off[s], op_off[s+1]) in order."""
    op_off: torch.Tensor   # (N+1,) int64
    kind: torch.Tensor     # (n_ops,) uint8: 0 = Op::Add, 1 = Op::Rm
    actor: torch.Tensor    # (n_ops,) int32  (Add: dot.actor)
    counter: torch.Tensor  # (n_ops,) int64  (Add: dot.counter, u64 bits)
    rm_row: torch.Tensor   # (n_ops,) int32  (Rm: row of rm_clock)
    rm_clock: torch.Tensor  # (n_rm, A) int64
    mem_off: torch.Tensor  # (n_ops+1,) int64
    mem: torch.Tensor      # (n_mem,) int32 member indices


def encode_ops(streams, A: int, device) -> OrswotOpBatch:
    """Host ingest of per-state op streams (already interned to dense indices).

    streams[s] is a sequence of ops, each ("add", actor, counter, members) for
    Op::Add { dot: Dot { actor, counter }, members } or ("rm", clock, members) for
    Op::Rm { clock, members }, with `clock` a mapping actor -> counter or a dense row of A
    counters and `members` an iterable of member indices (orswot.rs:33-46)."""
    op_off, kind, actor, counter, rm_row, mem_off, mem, rm_rows = [0], [], [], [], [], [0], [], []
    for ops in streams:
        for op in ops:
            if op[0] == "add":
                _, a, k, ms = op
                kind.append(0)
                actor.append(int(a))
                counter.append(int(k))
                rm_row.append(0)
            elif op[0] == "rm":
                _, clk, ms = op
                row = np.zeros(A, dtype=np.uint64)
                if hasattr(clk, "items"):
                    for a, k in clk.items():
                        row[int(a)] = np.uint64(k)
                else:
                    row[:] = np.asarray(clk, dtype=np.uint64)
                kind.append(1)
                actor.append(0)
                counter.append(0)
                rm_row.append(len(rm_rows))
                rm_rows.append(row)
            else:
                raise ValueError(f"orswot.encode_ops: unknown op {op[0]!r}")
            ms = [int(m) for m in ms]
            mem.extend(ms)
            mem_off.append(len(mem))
        op_off.append(len(kind))

    def t(x, dt):
        return torch.from_numpy(np.asarray(x, dtype=dt)).to(device)

    n_rm = len(rm_rows)
    rm_rows.append(np.zeros(A, dtype=np.uint64))  # pads: never-empty device buffers (rm_clock, mem)
    mem.append(0)
    rc = np.array(rm_rows, dtype=np.uint64).reshape(n_rm + 1, A)
    return OrswotOpBatch(
        t(op_off, np.int64), t(kind, np.uint8), t(actor, np.int32),
        t(np.array(counter, dtype=np.uint64).view(np.int64), np.int64), t(rm_row, np.int32),
        torch.from_numpy(rc.view(np.int64)).to(device), t(mem_off, np.int64), t(mem, np.int32))


def apply_batch(clock: torch.Tensor, entries: torch.Tensor, def_clock: torch.Tensor, def_members: torch.Tensor,
                def_count: torch.Tensor, ops: OrswotOpBatch, ctx: Optional[Context] = None) -> torch.Tensor:
    """Apply every state's op stream in place (clock (N, A), entries (N, M, A), deferred slots
    def_clock (N, Dcap, A) / def_members (N, Dcap, ceil(M/64)) / def_count (N,) int32).
    Returns the per-state status (N,) int32 tensor (include/crdt_gpu.h: bit 0 = deferred
    capacity exceeded, bit 1 = out-of-range op skipped, bits 2-3 = invalid input, state untouched)."""
    ctx = ctx or Context.default(clock.device.index)
    for t, nm in ((clock, "clock"), (entries, "entries"), (def_clock, "def_clock"), (def_members, "def_members")):
        ctx.check_tensor(t, f"orswot.apply_batch({nm})")
    if clock.dim() != 2 or entries.dim() != 3 or def_clock.dim() != 3 or def_members.dim() != 3:
        raise ValueError("orswot.apply_batch: clock (N,A), entries (N,M,A), def_clock (N,Dcap,A), "
                         "def_members (N,Dcap,Mw) expected")
    N, A = clock.shape
    M = entries.shape[1]
    Mw = (M + 63) // 64
    Dcap = def_clock.shape[1]
    if (entries.shape[0] != N or entries.shape[2] != A or clock.stride(1) != 1 or entries.stride(2) != 1
            or entries.stride(0) < M * entries.stride(1)):
        raise ValueError(f"orswot.apply_batch: entries {tuple(entries.shape)} / clock {tuple(clock.shape)} mismatch")
    if (tuple(def_clock.shape) != (N, Dcap, A) or tuple(def_members.shape) != (N, Dcap, Mw)
            or not def_clock.is_contiguous() or not def_members.is_contiguous()):
        raise ValueError("orswot.apply_batch: def_clock / def_members must be contiguous (N, Dcap, A) / (N, Dcap, Mw)")
    if def_count.dtype not in (torch.int32, torch.uint32) or tuple(def_count.shape) != (N,):
        raise ValueError("orswot.apply_batch: def_count must be an (N,) int32 tensor")
    if ops.op_off.shape[0] != N + 1:
        raise ValueError(f"orswot.apply_batch: op_off has {ops.op_off.shape[0]} entries, expected {N + 1}")
    want = {"op_off": (torch.int64, torch.uint64), "kind": (torch.uint8,), "actor": (torch.int32, torch.uint32),
            "counter": (torch.int64, torch.uint64), "rm_row": (torch.int32, torch.uint32),
            "rm_clock": (torch.int64, torch.uint64), "mem_off": (torch.int64, torch.uint64),
            "mem": (torch.int32, torch.uint32)}
    for nm, t in list(zip(ops._fields, ops)) + [("def_count", def_count)]:
        dts = want.get(nm, (torch.int32, torch.uint32))
        if t.device.type != "cuda" or t.device.index != ctx.device:
            raise ValueError(f"orswot.apply_batch({nm}): expected a cuda:{ctx.device} tensor")
        if t.dtype not in dts or not t.is_contiguous():
            raise ValueError(f"orswot.apply_batch({nm}): expected a contiguous tensor of {dts}")
    if ops.mem_off.shape[0] < ops.kind.shape[0] + 1 or ops.rm_clock.dim() != 2 or ops.rm_clock.shape[1] != A:
        raise ValueError("orswot.apply_batch: mem_off needs n_ops+1 entries, rm_clock (n_rm, A)")
    for nm in ("actor", "counter", "rm_row"):
        if getattr(ops, nm).shape[0] != ops.kind.shape[0]:
            raise ValueError(f"orswot.apply_batch: ops.{nm} must have n_ops entries")
    st = _abi.OrswotStates()
    st.N, st.M, st.A, st.Dcap = N, M, A, Dcap
    st.clock, st.clock_stride = clock.data_ptr(), clock.stride(0)
    st.entries, st.entry_mstride, st.entry_sstride = entries.data_ptr(), entries.stride(1), entries.stride(0)
    st.def_clock, st.def_members, st.def_count = def_clock.data_ptr(), def_members.data_ptr(), def_count.data_ptr()
    o = _abi.OrswotOps()
    o.n_ops = ops.kind.shape[0]
    o.op_off, o.kind, o.actor, o.counter = (ops.op_off.data_ptr(), ops.kind.data_ptr(), ops.actor.data_ptr(),
                                            ops.counter.data_ptr())
    o.rm_row, o.rm_clock, o.n_rm_rows = ops.rm_row.data_ptr(), ops.rm_clock.data_ptr(), ops.rm_clock.shape[0]
    o.mem_off, o.mem, o.n_mem = ops.mem_off.data_ptr(), ops.mem.data_ptr(), ops.mem.shape[0]
    status = torch.empty(N, dtype=torch.int32, device=clock.device)
    ctx.call("crdt_orswot_apply_batch", ctypes.byref(st), ctypes.byref(o), dptr(status))
    return status


def deferred_slots(def_clock: torch.Tensor, def_members: torch.Tensor, def_count: torch.Tensor, s: int) -> set:
    """Egress of state s's deferred list to {(rm clock tuple, frozenset of members)}."""
    n = int(def_count[s].item())
    keep = torch.ones(n, dtype=torch.uint8)
    return deferred_set(def_clock[s, :n], keep, def_members[s, :n])


def _forget_clock(ctx, y, N, A, what):
    ctx.check_tensor(y, what)
    if y.dim() == 1:
        if y.shape[0] != A:
            raise ValueError(f"{what}: y must be (A,) or (N, A)")
        return y, 0
    if tuple(y.shape) != (N, A) or y.stride(1) != 1:
        raise ValueError(f"{what}: y must be (A,) or (N, A) with contiguous rows")
    return y, y.stride(0)


def _forget_deferred(ctx, def_clock, def_state, N, A, what):
    """-> (ptr, state ptr, D, keep tensor or None)"""
    if def_clock is None or def_clock.shape[0] == 0:
        return None, None, 0, None
    ctx.check_tensor(def_clock, what)
    D = def_clock.shape[0]
    if tuple(def_clock.shape) != (D, A) or not def_clock.is_contiguous():
        raise ValueError(f"{what}: def_clock must be a contiguous (D, A) tensor")
    if (def_state is None or def_state.dtype not in (torch.int32, torch.uint32) or tuple(def_state.shape) != (D,)
            or def_state.device != def_clock.device or not def_state.is_contiguous()):
        raise ValueError(f"{what}: def_state must be a contiguous (D,) int32 tensor on the same device")
    keep = torch.empty(D, dtype=torch.uint8, device=def_clock.device)
    return def_clock.data_ptr(), def_state.data_ptr(), D, keep


def forget_batch(clock: torch.Tensor, entries: torch.Tensor, y: torch.Tensor, def_clock: Optional[torch.Tensor] = None,
                 def_state: Optional[torch.Tensor] = None, ctx: Optional[Context] = None) -> Optional[torch.Tensor]:
    """Causal::forget of N Orswot states in place (orswot.rs:150-183): clock (N, A), entries
    (N, M, A), y (A,) shared or (N, A) per state, deferred rm clocks def_clock (D, A) of states
    def_state (D,) int32.  Returns def_keep (D,) uint8 (0 = that remove was forgotten) or None."""
    ctx = ctx or Context.default(clock.device.index)
    ctx.check_tensor(clock, "orswot.forget_batch(clock)")
    ctx.check_tensor(entries, "orswot.forget_batch(entries)")
    if clock.dim() != 2 or entries.dim() != 3 or clock.stride(1) != 1 or entries.stride(2) != 1:
        raise ValueError("orswot.forget_batch: clock (N, A), entries (N, M, A) with the actor axis contiguous")
    N, A = clock.shape
    M = entries.shape[1]
    if entries.shape[0] != N or entries.shape[2] != A:
        raise ValueError("orswot.forget_batch: entries do not match clock")
    y, ys = _forget_clock(ctx, y, N, A, "orswot.forget_batch(y)")
    dp, sp, D, keep = _forget_deferred(ctx, def_clock, def_state, N, A, "orswot.forget_batch(def_clock)")
    ctx.call("crdt_orswot_forget_batch", clock.data_ptr(), clock.stride(0), entries.data_ptr(), entries.stride(1),
             entries.stride(0), N, M, A, y.data_ptr(), ys, dp, sp, D, keep.data_ptr() if keep is not None else None)
    return keep


# ---------------------------------------------------------------------------------------------
# Pairwise in-place merge_batch: self[i].merge(other[i]) (orswot.rs:81-149)
# ---------------------------------------------------------------------------------------------
class OrswotStates(NamedTuple):
    """N Orswot states in the per-state layout of apply_batch / merge_batch."""
    clock: torch.Tensor        # (N, A)
    entries: torch.Tensor      # (N, M, A)
    def_clock: torch.Tensor    # (N, Dcap, A)
    def_members: torch.Tensor  # (N, Dcap, ceil(M/64))
    def_count: torch.Tensor    # (N,) int32


def _states_struct(ctx: Context, st: OrswotStates, what: str) -> "_abi.OrswotStates":
    for t, nm in ((st.clock, "clock"), (st.entries, "entries"), (st.def_clock, "def_clock"),
                  (st.def_members, "def_members")):
        ctx.check_tensor(t, f"{what}({nm})")
    if st.clock.dim() != 2 or st.entries.dim() != 3 or st.def_clock.dim() != 3 or st.def_members.dim() != 3:
        raise ValueError(f"{what}: clock (N,A), entries (N,M,A), def_clock (N,Dcap,A), def_members (N,Dcap,Mw)")
    N, A = st.clock.shape
    M = st.entries.shape[1]
    Dcap = st.def_clock.shape[1]
    if (st.entries.shape[0] != N or st.entries.shape[2] != A or st.clock.stride(1) != 1 or st.entries.stride(2) != 1
            or st.entries.stride(0) < M * st.entries.stride(1)):
        raise ValueError(f"{what}: entries {tuple(st.entries.shape)} / clock {tuple(st.clock.shape)} mismatch")
    if (tuple(st.def_clock.shape) != (N, Dcap, A) or tuple(st.def_members.shape) != (N, Dcap, (M + 63) // 64)
            or not st.def_clock.is_contiguous() or not st.def_members.is_contiguous()):
        raise ValueError(f"{what}: def_clock / def_members must be contiguous (N, Dcap, A) / (N, Dcap, Mw)")
    if (st.def_count.dtype not in (torch.int32, torch.uint32) or tuple(st.def_count.shape) != (N,)
            or st.def_count.device != st.clock.device):
        raise ValueError(f"{what}: def_count must be an (N,) int32 tensor on the states' device")
    s = _abi.OrswotStates()
    s.N, s.M, s.A, s.Dcap = N, M, A, Dcap
    s.clock, s.clock_stride = st.clock.data_ptr(), st.clock.stride(0)
    s.entries, s.entry_mstride, s.entry_sstride = st.entries.data_ptr(), st.entries.stride(1), st.entries.stride(0)
    s.def_clock, s.def_members, s.def_count = st.def_clock.data_ptr(), st.def_members.data_ptr(), st.def_count.data_ptr()
    return s


def merge_batch(self_states: OrswotStates, other: OrswotStates, ctx: Optional[Context] = None) -> torch.Tensor:
    """self[i].merge(other[i]) for every i, in place on `self_states` (CvRDT::merge, traits.rs:4-7 ->
    Orswot::merge, orswot.rs:81-149), exact for any pair of states.  Returns status (N,) int32:
    bit 0 = more surviving deferred removes than self's Dcap slots, bit 2 = invalid def_count."""
    ctx = ctx or Context.default(self_states.clock.device.index)
    a = _states_struct(ctx, self_states, "orswot.merge_batch(self)")
    b = _states_struct(ctx, other, "orswot.merge_batch(other)")
    if (a.N, a.M, a.A) != (b.N, b.M, b.A):
        raise ValueError("orswot.merge_batch: self and other differ in N, M or A")
    status = torch.empty(a.N, dtype=torch.int32, device=self_states.clock.device)
    ctx.call("crdt_orswot_merge_batch", ctypes.byref(a), ctypes.byref(b), dptr(status))
    return status
