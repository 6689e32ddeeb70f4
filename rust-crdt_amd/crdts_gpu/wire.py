"""Serde wire format ingest / egress on the device (include/crdt_gpu.h "serde wire format").

Replicas ship whole serialized states; these calls turn a batch of received frames (the bytes
`bincode::serialize` writes for VClock / GCounter / PNCounter<u32>, GSet<u64>, LWWReg<u64, u64>,
Orswot<u64, u32>) into the dense layout the merge kernels read, and merged dense states back into
frames.  Every tensor is a device tensor: bytes (uint8), frame offsets (int64, N+1, 4-byte
aligned), dictionaries (sorted ascending: actors int32 holding u32 ids, members / elements int64
holding u64 ids).  Nothing here runs on the host except the shape checks.

    rows, status = vclock_ingest(bytes, frame_off, actors)          # (N, A), (N,) int32
    frame_off, data = vclock_egress(rows, actors)                   # (N+1,), (total,) uint8
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple, Optional

import torch

from .context import Context, dptr

BAD, MISSING, CAP = 1, 2, 4  # status bits


def _ctx(t: torch.Tensor, ctx: Optional[Context]) -> Context:
    return ctx or Context.default(t.device.index)


def _frames(ctx, data, frame_off, what):
    ctx.check_tensor(data, f"{what}(bytes)", (torch.uint8,))
    ctx.check_tensor(frame_off, f"{what}(frame_off)")
    if data.dtype != torch.uint8 or data.dim() != 1 or not data.is_contiguous():
        raise ValueError(f"{what}: bytes must be a contiguous uint8 vector")
    if frame_off.dtype != torch.int64 or frame_off.dim() != 1 or not frame_off.is_contiguous() or frame_off.shape[0] < 1:
        raise ValueError(f"{what}: frame_off must be a contiguous int64 (N+1,) tensor")
    return frame_off.shape[0] - 1


def _dict(ctx, d, dt, what):
    ctx.check_tensor(d, what, (dt,))
    if d.dtype != dt or d.dim() != 1 or not d.is_contiguous() or d.shape[0] == 0:
        raise ValueError(f"{what}: a non-empty contiguous {dt} dictionary is required")
    return d.shape[0]


def _status(N, dev):
    return torch.zeros(N, dtype=torch.int32, device=dev)


def _ptr_or_dummy(data):
    return dptr(data) if data.numel() else None


def vclock_ingest(data: torch.Tensor, frame_off: torch.Tensor, actors: torch.Tensor, out: Optional[torch.Tensor] = None,
                  ctx: Optional[Context] = None, _fn: str = "crdt_vclock_ingest", _k: int = 1):
    """VClock / GCounter frames -> (rows (N, A) int64, status (N,) int32)."""
    ctx = _ctx(data, ctx)
    N = _frames(ctx, data, frame_off, "wire.vclock_ingest")
    A = _dict(ctx, actors, torch.int32, "wire.vclock_ingest(actors)")
    if out is None:
        out = torch.empty((N, _k * A), dtype=torch.int64, device=data.device)
    if out.dim() != 2 or out.shape[0] != N or out.shape[1] < _k * A or out.stride(1) != 1:
        raise ValueError(f"wire ingest: out must be ({N}, >= {_k * A}) with contiguous rows")
    st = _status(N, data.device)
    ctx.call(_fn, _ptr_or_dummy(data), dptr(frame_off), N, dptr(actors), A, dptr(out), out.stride(0), dptr(st))
    return out, st


def pncounter_ingest(data, frame_off, actors, out=None, ctx=None):
    """PNCounter frames (p then n) -> (rows (N, 2A) = P | N, status)."""
    return vclock_ingest(data, frame_off, actors, out, ctx, "crdt_pncounter_ingest", 2)


def gset_ingest(data: torch.Tensor, frame_off: torch.Tensor, elems: torch.Tensor, out: Optional[torch.Tensor] = None,
                ctx: Optional[Context] = None):
    """GSet<u64> frames -> (bitmap rows (N, ceil(U/64)), status)."""
    ctx = _ctx(data, ctx)
    N = _frames(ctx, data, frame_off, "wire.gset_ingest")
    U = _dict(ctx, elems, torch.int64, "wire.gset_ingest(elems)")
    W = (U + 63) // 64
    if out is None:
        out = torch.empty((N, W), dtype=torch.int64, device=data.device)
    st = _status(N, data.device)
    ctx.call("crdt_gset_ingest", _ptr_or_dummy(data), dptr(frame_off), N, dptr(elems), U, dptr(out), out.stride(0),
             dptr(st))
    return out, st


def lwwreg_ingest(data: torch.Tensor, frame_off: torch.Tensor, ctx: Optional[Context] = None):
    """LWWReg<u64, u64> frames -> (marker (N,), val (N,), status)."""
    ctx = _ctx(data, ctx)
    N = _frames(ctx, data, frame_off, "wire.lwwreg_ingest")
    m = torch.empty(N, dtype=torch.int64, device=data.device)
    v = torch.empty_like(m)
    st = _status(N, data.device)
    ctx.call("crdt_lwwreg_ingest", _ptr_or_dummy(data), dptr(frame_off), N, dptr(m), dptr(v), dptr(st))
    return m, v, st


class OrswotFrames(NamedTuple):
    clock: torch.Tensor        # (N, A)
    entries: torch.Tensor      # (N, M, A)
    def_off: torch.Tensor      # (N+1,) int64, device: state s owns removes [def_off[s], def_off[s+1])
    def_clock: torch.Tensor    # (D, A)
    def_members: torch.Tensor  # (D, ceil(M/64))
    status: torch.Tensor       # (N,) int32


def orswot_ingest(data: torch.Tensor, frame_off: torch.Tensor, actors: torch.Tensor, members: torch.Tensor,
                  def_cap: Optional[int] = None, ctx: Optional[Context] = None) -> OrswotFrames:
    """Orswot<u64, u32> frames -> dense states + the deferred removes pooled in state order."""
    ctx = _ctx(data, ctx)
    N = _frames(ctx, data, frame_off, "wire.orswot_ingest")
    A = _dict(ctx, actors, torch.int32, "wire.orswot_ingest(actors)")
    M = _dict(ctx, members, torch.int64, "wire.orswot_ingest(members)")
    Mw = (M + 63) // 64
    dev = data.device
    clock = torch.empty((N, A), dtype=torch.int64, device=dev)
    entries = torch.empty((N, M, A), dtype=torch.int64, device=dev)
    def_off = torch.empty(N + 1, dtype=torch.int64, device=dev)
    cap = def_cap if def_cap is not None else max(1, N)
    dcl = torch.empty((cap, A), dtype=torch.int64, device=dev)
    dmb = torch.empty((cap, Mw), dtype=torch.int64, device=dev)
    st = _status(N, dev)
    nd = ctypes.c_size_t()
    ctx.call("crdt_orswot_ingest", _ptr_or_dummy(data), dptr(frame_off), N, dptr(actors), A, dptr(members), M,
             dptr(clock), dptr(entries), dptr(def_off), dptr(dcl), dptr(dmb), cap, ctypes.byref(nd), dptr(st))
    D = nd.value
    if D > cap and def_cap is None:  # more removes than guessed: once more with exactly enough room
        return orswot_ingest(data, frame_off, actors, members, def_cap=D, ctx=ctx)
    return OrswotFrames(clock, entries, def_off, dcl[:min(D, cap)], dmb[:min(D, cap)], st)


def _egress(ctx, fn, N, dev, *args):
    frame_off = torch.empty(N + 1, dtype=torch.int64, device=dev)
    total = ctypes.c_size_t()
    ctx.call(fn, *args, dptr(frame_off), None, 0, ctypes.byref(total))
    data = torch.empty(max(total.value, 1), dtype=torch.uint8, device=dev)
    ctx.call(fn, *args, dptr(frame_off), dptr(data), data.numel(), ctypes.byref(total))
    return frame_off, data[:total.value]


def vclock_egress(rows: torch.Tensor, actors: torch.Tensor, ctx: Optional[Context] = None, _fn="crdt_vclock_egress",
                  _k: int = 1):
    """Dense rows (N, A) -> (frame_off (N+1,), bytes) of VClock / GCounter frames."""
    ctx = _ctx(rows, ctx)
    ctx.check_tensor(rows, "wire.vclock_egress(rows)")
    A = _dict(ctx, actors, torch.int32, "wire.vclock_egress(actors)")
    if rows.dim() != 2 or rows.shape[1] < _k * A or rows.stride(1) != 1:
        raise ValueError(f"wire egress: rows must be (N, >= {_k * A}) with contiguous rows")
    N = rows.shape[0]
    return _egress(ctx, _fn, N, rows.device, dptr(rows), N, A, rows.stride(0), dptr(actors))


def pncounter_egress(rows, actors, ctx=None):
    return vclock_egress(rows, actors, ctx, "crdt_pncounter_egress", 2)


def gset_egress(rows: torch.Tensor, elems: torch.Tensor, ctx: Optional[Context] = None):
    ctx = _ctx(rows, ctx)
    ctx.check_tensor(rows, "wire.gset_egress(rows)")
    U = _dict(ctx, elems, torch.int64, "wire.gset_egress(elems)")
    if rows.dim() != 2 or rows.shape[1] < (U + 63) // 64 or rows.stride(1) != 1:
        raise ValueError("wire.gset_egress: rows must be (N, >= ceil(U/64))")
    N = rows.shape[0]
    return _egress(ctx, "crdt_gset_egress", N, rows.device, dptr(rows), N, U, rows.stride(0), dptr(elems))


def lwwreg_egress(marker: torch.Tensor, val: torch.Tensor, ctx: Optional[Context] = None):
    ctx = _ctx(marker, ctx)
    N = marker.shape[0]
    data = torch.empty(max(16 * N, 1), dtype=torch.uint8, device=marker.device)
    ctx.call("crdt_lwwreg_egress", dptr(marker.contiguous()), dptr(val.contiguous()), N, dptr(data))
    off = torch.arange(0, 16 * (N + 1), 16, dtype=torch.int64, device=marker.device)
    return off, data[:16 * N]


def orswot_egress(clock: torch.Tensor, entries: torch.Tensor, actors: torch.Tensor, members: torch.Tensor,
                  def_off: Optional[torch.Tensor] = None, def_clock: Optional[torch.Tensor] = None,
                  def_members: Optional[torch.Tensor] = None, def_keep: Optional[torch.Tensor] = None,
                  ctx: Optional[Context] = None):
    """Dense Orswot states (clock (N, A), entries (N, M, A)) + removes pooled by state (device
    def_off (N+1,), def_clock, def_members, def_keep or None) -> (frame_off, bytes)."""
    ctx = _ctx(clock, ctx)
    A = _dict(ctx, actors, torch.int32, "wire.orswot_egress(actors)")
    M = _dict(ctx, members, torch.int64, "wire.orswot_egress(members)")
    N = clock.shape[0]
    if tuple(clock.shape) != (N, A) or tuple(entries.shape) != (N, M, A) or not clock.is_contiguous() \
            or not entries.is_contiguous():
        raise ValueError("wire.orswot_egress: clock (N, A) and entries (N, M, A), contiguous")
    dp = [None, None, None, None]
    if def_off is not None:
        dp = [dptr(def_off), dptr(def_clock), dptr(def_members), dptr(def_keep) if def_keep is not None else None]
    return _egress(ctx, "crdt_orswot_egress", N, clock.device, dptr(clock), dptr(entries), N, M, A, dptr(actors),
                   dptr(members), *dp)


def map_ingest(data: torch.Tensor, frame_off: torch.Tensor, actors: torch.Tensor, keys: torch.Tensor, V: int,
               Dcap: int, ctx: Optional[Context] = None):
    """Map<u32, MVReg<u64>> frames -> (map.MapStates with V value slots per key and Dcap deferred
    slots per state, status (N,) int32).  keys: sorted u32 key dictionary (int32 tensor)."""
    from .map import MapStates, _map_states_structs
    ctx = _ctx(data, ctx)
    N = _frames(ctx, data, frame_off, "wire.map_ingest")
    A = _dict(ctx, actors, torch.int32, "wire.map_ingest(actors)")
    K = _dict(ctx, keys, torch.int32, "wire.map_ingest(keys)")
    dev = data.device
    z = lambda *shape: torch.zeros(shape, dtype=torch.int64, device=dev)  # noqa: E731
    st = MapStates(z(N, A), z(N, K, A), z(N, K, V, A), z(N, K, V), z(N, max(Dcap, 0), A), z(N, max(Dcap, 0), (K + 63) // 64),
                   torch.zeros(N, dtype=torch.int32, device=dev))
    s, d = _map_states_structs(ctx, st, "wire.map_ingest")
    status = _status(N, dev)
    ctx.call("crdt_map_ingest", _ptr_or_dummy(data), dptr(frame_off), dptr(actors), dptr(keys), ctypes.byref(s),
             ctypes.byref(d), dptr(status))
    return st, status


def map_egress(states, actors: torch.Tensor, keys: torch.Tensor, ctx: Optional[Context] = None):
    """map.MapStates (packed per-state blocks, deferred slots) -> (frame_off (N+1,), bytes)."""
    from .map import _map_states_structs
    ctx = _ctx(states.clock, ctx)
    _dict(ctx, actors, torch.int32, "wire.map_egress(actors)")
    _dict(ctx, keys, torch.int32, "wire.map_egress(keys)")
    s, d = _map_states_structs(ctx, states, "wire.map_egress")
    return _egress(ctx, "crdt_map_egress", states.clock.shape[0], states.clock.device, ctypes.byref(s), ctypes.byref(d),
                   dptr(actors), dptr(keys))


# ---- the value-typed Maps (round 5) ---------------------------------------------------------------
class MapCounterFrames(NamedTuple):
    """Map<u32, GCounter / PNCounter> states in the crdt_map_counter_states layout + deferred slots."""
    clock: torch.Tensor      # (N, A)
    ec: torch.Tensor         # (N, K, A)
    val: torch.Tensor        # (N, K, W, A)
    def_clock: torch.Tensor  # (N, Dcap, A)
    def_keys: torch.Tensor   # (N, Dcap, Kw)
    def_count: torch.Tensor  # (N,) int32


class MapOrswotFrames(NamedTuple):
    """Map<u32, Orswot<u64>> states in the crdt_map_orswot_states layout (the field names of
    map.MapOrswotLub, so map.orswot_apply_batch / orswot_forget_batch take it) + deferred slots."""
    clock: torch.Tensor      # (N, A)
    ec: torch.Tensor         # (N, K, A)
    oc: torch.Tensor         # (N, K, A)
    ent: torch.Tensor        # (N, K, M, A)
    vd_n: torch.Tensor       # (N, K) int32
    vd_clock: torch.Tensor   # (N, K, Vd, A)  (Vd nested slots per key, 16 by default)
    vd_mem: torch.Tensor     # (N, K, Vd) member bitmasks ((N, K, Vd, Mw) past M = 64)
    def_clock: torch.Tensor  # (N, Dcap, A)
    def_keys: torch.Tensor   # (N, Dcap, Kw)
    def_count: torch.Tensor  # (N,) int32


class MapNestedFrames(NamedTuple):
    """Map<u32, Map<u32, MVReg<u64>>> states in the crdt_map_nested_states layout (the field names of
    map.MapNestedLub, so map.nested_apply_batch / nested_forget_batch take it) + deferred slots."""
    clock: torch.Tensor      # (N, A)
    ec: torch.Tensor         # (N, K, A)
    ic: torch.Tensor         # (N, K, A)
    iec: torch.Tensor        # (N, K, K2, A)
    ivc: torch.Tensor        # (N, K, K2, Vs, A)  (Vs MVReg slots per inner key, 8 by default)
    ivv: torch.Tensor        # (N, K, K2, Vs)
    nval: torch.Tensor       # (N, K, K2) int32
    id_n: torch.Tensor       # (N, K) int32
    id_clock: torch.Tensor   # (N, K, Id, A)  (Id inner deferred slots per key, 16 by default)
    id_keys: torch.Tensor    # (N, K, 16) ((N, K, 16, K2w) mask words past K2 = 64)
    def_clock: torch.Tensor  # (N, Dcap, A)
    def_keys: torch.Tensor   # (N, Dcap, Kw)
    def_count: torch.Tensor  # (N,) int32


def _vmap_deferred(st):
    from . import _abi
    d = _abi.MapDeferred()
    Dcap = st.def_clock.shape[1]
    d.clock = dptr(st.def_clock) if Dcap else None
    d.keys = dptr(st.def_keys) if Dcap else None
    d.count = dptr(st.def_count)
    d.Dcap = Dcap
    return d


def _vmap_check(ctx, st, what):
    for nm, t in st._asdict().items():
        ctx.check_tensor(t, f"{what}({nm})", (torch.int32,) if nm in ("vd_n", "def_count", "nval", "id_n") else None)
        if not t.is_contiguous():
            raise ValueError(f"{what}: {nm} must be contiguous")
    N, A = st.clock.shape
    Dcap = st.def_clock.shape[1]
    K = st.ec.shape[1]
    if tuple(st.def_clock.shape) != (N, Dcap, A) or tuple(st.def_keys.shape) != (N, Dcap, (K + 63) // 64) \
            or tuple(st.def_count.shape) != (N,) or st.def_count.dtype != torch.int32:
        raise ValueError(f"{what}: deferred slots must be (N, Dcap, A), (N, Dcap, ceil(K/64)), (N,) int32")
    return N, K, A


def _counter_struct(ctx, st, what):
    from . import _abi
    N, K, A = _vmap_check(ctx, st, what)
    W = st.val.shape[2]
    if tuple(st.ec.shape) != (N, K, A) or tuple(st.val.shape) != (N, K, W, A) or W not in (1, 2):
        raise ValueError(f"{what}: clock (N, A), ec (N, K, A), val (N, K, W, A) with W = 1 or 2 expected")
    s = _abi.MapCounterStates()
    s.N, s.K, s.A, s.W = N, K, A, W
    s.clock, s.clock_stride = dptr(st.clock), A
    s.ec, s.ec_stride = dptr(st.ec), K * A
    s.val, s.val_stride = dptr(st.val), K * W * A
    return s, _vmap_deferred(st)


def _orswot_struct(ctx, st, what):
    from . import _abi
    N, K, A = _vmap_check(ctx, st, what)
    M = st.ent.shape[2]
    Mw = (M + 63) // 64
    Vd = st.vd_clock.shape[2] if st.vd_clock.dim() == 4 else 0
    vm = (N, K, Vd) if Mw == 1 else (N, K, Vd, Mw)
    if (tuple(st.oc.shape) != (N, K, A) or tuple(st.ent.shape) != (N, K, M, A) or tuple(st.vd_n.shape) != (N, K)
            or Vd < 16 or tuple(st.vd_clock.shape) != (N, K, Vd, A) or tuple(st.vd_mem.shape) != vm):
        raise ValueError(f"{what}: the crdt_map_orswot_states shapes expected")
    s = _abi.MapOrswotStates()
    s.N, s.K, s.M, s.A, s.Vd = N, K, M, A, Vd
    s.clock, s.ec, s.oc, s.ent = dptr(st.clock), dptr(st.ec), dptr(st.oc), dptr(st.ent)
    s.vd_n, s.vd_clock, s.vd_mem = dptr(st.vd_n), dptr(st.vd_clock), dptr(st.vd_mem)
    return s, _vmap_deferred(st)


def map_counter_ingest(data: torch.Tensor, frame_off: torch.Tensor, actors: torch.Tensor, keys: torch.Tensor,
                       W: int, Dcap: int, ctx: Optional[Context] = None):
    """Map<u32, GCounter<u32>> (W = 1) / Map<u32, PNCounter<u32>> (W = 2) frames ->
    (MapCounterFrames, status (N,) int32); keys: sorted u32 key dictionary (int32 tensor)."""
    ctx = _ctx(data, ctx)
    N = _frames(ctx, data, frame_off, "wire.map_counter_ingest")
    A = _dict(ctx, actors, torch.int32, "wire.map_counter_ingest(actors)")
    K = _dict(ctx, keys, torch.int32, "wire.map_counter_ingest(keys)")
    dev = data.device
    z = lambda *shape: torch.zeros(shape, dtype=torch.int64, device=dev)  # noqa: E731
    st = MapCounterFrames(z(N, A), z(N, K, A), z(N, K, W, A), z(N, Dcap, A), z(N, Dcap, (K + 63) // 64),
                          torch.zeros(N, dtype=torch.int32, device=dev))
    s, d = _counter_struct(ctx, st, "wire.map_counter_ingest")
    status = _status(N, dev)
    ctx.call("crdt_map_counter_ingest", _ptr_or_dummy(data), dptr(frame_off), dptr(actors), dptr(keys),
             ctypes.byref(s), ctypes.byref(d), dptr(status))
    return st, status


def map_counter_egress(states: MapCounterFrames, actors: torch.Tensor, keys: torch.Tensor,
                       ctx: Optional[Context] = None):
    """MapCounterFrames -> (frame_off (N+1,), bytes)."""
    ctx = _ctx(states.clock, ctx)
    _dict(ctx, actors, torch.int32, "wire.map_counter_egress(actors)")
    _dict(ctx, keys, torch.int32, "wire.map_counter_egress(keys)")
    s, d = _counter_struct(ctx, states, "wire.map_counter_egress")
    return _egress(ctx, "crdt_map_counter_egress", states.clock.shape[0], states.clock.device, ctypes.byref(s),
                   ctypes.byref(d), dptr(actors), dptr(keys))


def map_orswot_ingest(data: torch.Tensor, frame_off: torch.Tensor, actors: torch.Tensor, keys: torch.Tensor,
                      members: torch.Tensor, Dcap: int, ctx: Optional[Context] = None, vd_cap: int = 16):
    """Map<u32, Orswot<u64, u32>> frames -> (MapOrswotFrames, status (N,) int32); members: sorted
    u64 member dictionary (int64 tensor); vd_cap nested deferred slots per key (>= 16)."""
    ctx = _ctx(data, ctx)
    N = _frames(ctx, data, frame_off, "wire.map_orswot_ingest")
    A = _dict(ctx, actors, torch.int32, "wire.map_orswot_ingest(actors)")
    K = _dict(ctx, keys, torch.int32, "wire.map_orswot_ingest(keys)")
    M = _dict(ctx, members, torch.int64, "wire.map_orswot_ingest(members)")
    dev = data.device
    Mw = (M + 63) // 64
    z = lambda *shape: torch.zeros(shape, dtype=torch.int64, device=dev)  # noqa: E731
    st = MapOrswotFrames(z(N, A), z(N, K, A), z(N, K, A), z(N, K, M, A),
                         torch.zeros((N, K), dtype=torch.int32, device=dev), z(N, K, vd_cap, A),
                         z(N, K, vd_cap) if Mw == 1 else z(N, K, vd_cap, Mw), z(N, Dcap, A), z(N, Dcap, (K + 63) // 64),
                         torch.zeros(N, dtype=torch.int32, device=dev))
    s, d = _orswot_struct(ctx, st, "wire.map_orswot_ingest")
    status = _status(N, dev)
    ctx.call("crdt_map_orswot_ingest", _ptr_or_dummy(data), dptr(frame_off), dptr(actors), dptr(keys),
             dptr(members), ctypes.byref(s), ctypes.byref(d), dptr(status))
    return st, status


def map_orswot_egress(states: MapOrswotFrames, actors: torch.Tensor, keys: torch.Tensor, members: torch.Tensor,
                      ctx: Optional[Context] = None):
    """MapOrswotFrames -> (frame_off (N+1,), bytes)."""
    ctx = _ctx(states.clock, ctx)
    _dict(ctx, actors, torch.int32, "wire.map_orswot_egress(actors)")
    _dict(ctx, keys, torch.int32, "wire.map_orswot_egress(keys)")
    _dict(ctx, members, torch.int64, "wire.map_orswot_egress(members)")
    s, d = _orswot_struct(ctx, states, "wire.map_orswot_egress")
    return _egress(ctx, "crdt_map_orswot_egress", states.clock.shape[0], states.clock.device, ctypes.byref(s),
                   ctypes.byref(d), dptr(actors), dptr(keys), dptr(members))


def _nested_struct(ctx, st, what):
    from . import _abi
    N, K, A = _vmap_check(ctx, st, what)
    K2 = st.iec.shape[2]
    K2w = (K2 + 63) // 64 if K2 > 64 else 1
    Id = st.id_clock.shape[2] if st.id_clock.dim() == 4 else 0
    if Id < 16:
        raise ValueError(f"{what}: id_clock (N, K, Id, A) with Id >= 16 expected")
    Vs = st.ivc.shape[3] if st.ivc.dim() == 5 else 0
    if not 8 <= Vs <= 64:
        raise ValueError(f"{what}: ivc (N, K, K2, Vs, A) with Vs in 8..64 expected")
    shapes = dict(ic=(N, K, A), iec=(N, K, K2, A), ivc=(N, K, K2, Vs, A), ivv=(N, K, K2, Vs), nval=(N, K, K2),
                  id_n=(N, K), id_clock=(N, K, Id, A), id_keys=(N, K, Id) if K2w == 1 else (N, K, Id, K2w))
    for nm, shp in shapes.items():
        if tuple(getattr(st, nm).shape) != shp:
            raise ValueError(f"{what}: {nm} must be {shp}")
    s = _abi.MapNestedStates()
    s.N, s.K, s.K2, s.A, s.Id, s.Vs = N, K, K2, A, Id, Vs
    for nm in ("clock", "ec", "ic", "iec", "ivc", "ivv", "nval", "id_n", "id_clock", "id_keys"):
        setattr(s, nm, dptr(getattr(st, nm)))
    return s, _vmap_deferred(st)


def map_nested_ingest(data: torch.Tensor, frame_off: torch.Tensor, actors: torch.Tensor, keys: torch.Tensor,
                      ikeys: torch.Tensor, Dcap: int, ctx: Optional[Context] = None, id_cap: int = 16,
                      v_cap: int = 8):
    """Map<u32, Map<u32, MVReg<u64>>> frames -> (MapNestedFrames, status (N,) int32); ikeys: sorted
    u32 inner-key dictionary (int32 tensor, at most 256; past 64 the inner key sets are K2w words)."""
    ctx = _ctx(data, ctx)
    N = _frames(ctx, data, frame_off, "wire.map_nested_ingest")
    A = _dict(ctx, actors, torch.int32, "wire.map_nested_ingest(actors)")
    K = _dict(ctx, keys, torch.int32, "wire.map_nested_ingest(keys)")
    K2 = _dict(ctx, ikeys, torch.int32, "wire.map_nested_ingest(ikeys)")
    dev = data.device
    z = lambda *shape: torch.zeros(shape, dtype=torch.int64, device=dev)  # noqa: E731
    z32 = lambda *shape: torch.zeros(shape, dtype=torch.int32, device=dev)  # noqa: E731
    st = MapNestedFrames(z(N, A), z(N, K, A), z(N, K, A), z(N, K, K2, A), z(N, K, K2, v_cap, A), z(N, K, K2, v_cap),
                         z32(N, K, K2), z32(N, K), z(N, K, id_cap, A),
                         z(N, K, id_cap) if K2 <= 64 else z(N, K, id_cap, (K2 + 63) // 64), z(N, Dcap, A),
                         z(N, Dcap, (K + 63) // 64), z32(N))
    s, d = _nested_struct(ctx, st, "wire.map_nested_ingest")
    status = _status(N, dev)
    ctx.call("crdt_map_nested_ingest", _ptr_or_dummy(data), dptr(frame_off), dptr(actors), dptr(keys), dptr(ikeys),
             ctypes.byref(s), ctypes.byref(d), dptr(status))
    return st, status


def map_nested_egress(states: MapNestedFrames, actors: torch.Tensor, keys: torch.Tensor, ikeys: torch.Tensor,
                      ctx: Optional[Context] = None):
    """MapNestedFrames -> (frame_off (N+1,), bytes)."""
    ctx = _ctx(states.clock, ctx)
    _dict(ctx, actors, torch.int32, "wire.map_nested_egress(actors)")
    _dict(ctx, keys, torch.int32, "wire.map_nested_egress(keys)")
    _dict(ctx, ikeys, torch.int32, "wire.map_nested_egress(ikeys)")
    s, d = _nested_struct(ctx, states, "wire.map_nested_egress")
    return _egress(ctx, "crdt_map_nested_egress", states.clock.shape[0], states.clock.device, ctypes.byref(s),
                   ctypes.byref(d), dptr(actors), dptr(keys), dptr(ikeys))
