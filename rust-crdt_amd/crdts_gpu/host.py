"""Host-memory entry points (crdt_mem_kind = CRDT_MEM_HOST, csrc/host_stage.hip).

The drop-in form a reference caller starts from: replicas in host memory, as
`CvRDT::merge` folded over a `Vec<Self>` (traits.rs:4-7) or `merge_batch(&mut [Self], Vec<Self>)`.
The arrays are numpy uint64 (u64 bit patterns, dense interned layout as for the device entry
points); the library streams them through two device chunk buffers, overlapping the PCIe copy of
one chunk with the HBM fold of the previous, and returns with the result in host memory.

A HostContext is a separate crdt_ctx switched to CRDT_MEM_HOST (the device-pointer Context of a
process stays in device mode).  `pinned_empty` gives page-locked arrays (crdt_host_alloc) that
the library copies by DMA without the runtime's pageable staging.
"""
from __future__ import annotations

import ctypes
import weakref
from typing import NamedTuple, Optional

import numpy as np

from . import _abi

_KINDS = {"vclock": ("crdt_vclock", 1), "gcounter": ("crdt_gcounter", 1), "pncounter": ("crdt_pncounter", 2),
          "gset": ("crdt_gset", 1)}


class HostContext:
    """A crdt_ctx in CRDT_MEM_HOST mode on HIP device `device`."""

    def __init__(self, device: int = 0, tune: Optional[str] = None):
        self.lib = _abi.load()
        ptr = ctypes.c_void_p()
        _abi.check(None, "crdt_ctx_create", self.lib.crdt_ctx_create(int(device), ctypes.byref(ptr)))
        self.ptr = ptr
        self.call("crdt_ctx_set_mem_kind", _abi.CRDT_MEM_HOST)
        if tune:
            self.call("crdt_ctx_tune", tune.encode())

    _by_device: dict = {}

    @classmethod
    def default(cls, device: int = 0) -> "HostContext":
        """One cached host-mode ctx per device for calls made without an explicit ctx (each ctx owns
        two stage_kb device chunk buffers and an accumulator: a fresh one per call would churn
        device memory until its finalizer ran)."""
        ctx = cls._by_device.get(int(device))
        if ctx is None or not getattr(ctx, "ptr", None):
            ctx = cls(device)
            cls._by_device[int(device)] = ctx
        return ctx

    def call(self, name: str, *args) -> None:
        _abi.check(self.ptr, name, getattr(self.lib, name)(self.ptr, *args))

    def raw(self, name: str, *args) -> int:
        """The status code itself (tests of the refusal paths)."""
        return int(getattr(self.lib, name)(self.ptr, *args))

    def close(self) -> None:
        if getattr(self, "ptr", None):
            self.lib.crdt_ctx_destroy(self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


def pinned_empty(shape, dtype=np.uint64) -> np.ndarray:
    """A numpy array in page-locked host memory (crdt_host_alloc), freed with the array."""
    lib = _abi.load()
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    p = ctypes.c_void_p()
    _abi.check(None, "crdt_host_alloc", lib.crdt_host_alloc(max(n, 1), ctypes.byref(p)))
    buf = (ctypes.c_char * max(n, 1)).from_address(p.value)
    arr = np.frombuffer(buf, dtype=dt, count=int(np.prod(shape))).reshape(shape)
    weakref.finalize(buf, lib.crdt_host_free, ctypes.c_void_p(p.value))
    return arr


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _u64(a: np.ndarray, what: str) -> np.ndarray:
    if not isinstance(a, np.ndarray) or a.dtype not in (np.uint64, np.int64):
        raise TypeError(f"{what}: expected a uint64 numpy array")
    return a


def _rows(a: np.ndarray, what: str):
    """(rows, W, row_stride) of a 2-D array with unit inner stride."""
    if a.ndim != 2 or a.strides[1] != 8 or a.strides[0] % 8:
        raise ValueError(f"{what}: need a 2-D array with contiguous rows")
    return a.shape[0], a.shape[1], a.strides[0] // 8


def lub_many(kind: str, replicas: np.ndarray, out: Optional[np.ndarray] = None, accumulate: bool = False,
             ctx: Optional[HostContext] = None) -> np.ndarray:
    """G folds over R host replicas: replicas (R, W) or (G, R, W) (W = A, 2A for pncounter,
    words for gset); rows may be strided views.  Returns (W,) or (G, W) in host memory."""
    prefix, wdiv = _KINDS[kind]
    ctx = ctx or HostContext.default()
    _u64(replicas, "replicas")
    squeeze = replicas.ndim == 2
    r3 = replicas[None] if squeeze else replicas
    if r3.size == 0:  # numpy gives empty arrays zero strides: any layout is fine (nothing is read)
        r3 = np.zeros(r3.shape, np.uint64)
    if r3.ndim != 3 or (r3.size and (r3.strides[2] != 8 or r3.strides[1] % 8 or r3.strides[0] % 8)):
        raise ValueError("lub_many: replicas must be (R, W) or (G, R, W) with contiguous rows")
    G, R, W = r3.shape
    if W % wdiv:
        raise ValueError(f"{kind}: row width {W} is not a multiple of {wdiv}")
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs out")
        out = np.zeros((W,) if squeeze else (G, W), np.uint64)
    o2 = out[None] if out.ndim == 1 else out
    _, Wo, ostride = _rows(o2, "out")
    if Wo != W or o2.shape[0] != G:
        raise ValueError("out shape mismatch")
    rs, gs = (r3.strides[1] // 8, r3.strides[0] // 8) if r3.size else (W, R * W)
    ctx.call(f"{prefix}_lub_many", _ptr(r3), G, R, W // wdiv, rs, gs, _ptr(o2),
             ostride, _abi.CRDT_ACCUMULATE if accumulate else 0)
    return out


def merge_batch(kind: str, self_rows: np.ndarray, other_rows: np.ndarray, ctx: Optional[HostContext] = None) -> np.ndarray:
    """self[i] := self[i] ⊔ other[i] over host rows (N, W), in place; returns self_rows."""
    prefix, wdiv = _KINDS[kind]
    ctx = ctx or HostContext.default()
    N, W, ss = _rows(_u64(self_rows, "self"), "self")
    N2, W2, os_ = _rows(_u64(other_rows, "other"), "other")
    if (N, W) != (N2, W2):
        raise ValueError("merge_batch: shape mismatch")
    ctx.call(f"{prefix}_merge_batch", _ptr(self_rows), _ptr(other_rows), N, W // wdiv, ss, os_)
    return self_rows


class LwwResult(NamedTuple):
    marker: np.ndarray
    val: np.ndarray
    first_conflict: np.ndarray  # UINT64_MAX where no merge of the fold errs


def lwwreg_lub_many(marker: np.ndarray, val: np.ndarray, ctx: Optional[HostContext] = None) -> LwwResult:
    """Folds of LWWReg::merge over host replicas: marker/val (R,) or (G, R) (crdt_lwwreg_lub_many)."""
    ctx = ctx or HostContext.default()
    m2 = _u64(marker, "marker")[None] if marker.ndim == 1 else marker
    v2 = _u64(val, "val")[None] if val.ndim == 1 else val
    if m2.shape != v2.shape or m2.strides != v2.strides or m2.strides[1] != 8:
        raise ValueError("lwwreg_lub_many: marker and val must share a shape with contiguous rows")
    G, R = m2.shape
    om, ov, fc = (np.zeros(G, np.uint64) for _ in range(3))
    ctx.call("crdt_lwwreg_lub_many", _ptr(m2), _ptr(v2), G, R, m2.strides[0] // 8, _ptr(om), _ptr(ov), _ptr(fc), 0)
    return LwwResult(om, ov, fc)


def lwwreg_merge_batch(self_marker: np.ndarray, self_val: np.ndarray, other_marker: np.ndarray, other_val: np.ndarray,
                       ctx: Optional[HostContext] = None) -> np.ndarray:
    """self[i].merge(other[i]) in place over host arrays; returns the (N,) uint8 conflict flags."""
    ctx = ctx or HostContext.default()
    arrs = [_u64(a, n) for a, n in ((self_marker, "self_marker"), (self_val, "self_val"),
                                     (other_marker, "other_marker"), (other_val, "other_val"))]
    N = arrs[0].shape[0]
    if any(a.shape != (N,) or a.strides != (8,) for a in arrs):
        raise ValueError("lwwreg_merge_batch: four contiguous (N,) arrays")
    conflict = np.zeros(N, np.uint8)
    ctx.call("crdt_lwwreg_merge_batch", *[_ptr(a) for a in arrs], N, _ptr(conflict))
    return conflict


class OrswotHostLub(NamedTuple):
    clock: np.ndarray        # (G, A)
    entries: np.ndarray      # (G, M, A)
    def_keep: np.ndarray     # (D,) uint8
    def_members: np.ndarray  # (D, Mw)


def orswot_lub_many(clock: np.ndarray, entries: np.ndarray, def_off=None, def_clock: Optional[np.ndarray] = None,
                    def_members: Optional[np.ndarray] = None, ctx: Optional[HostContext] = None) -> OrswotHostLub:
    """crdt_orswot_lub_many on host arrays: clock (G, R, A), entries (G, R, M, A) (or without G),
    deferred removes pooled per group (def_off G+1, def_clock (D, A), def_members (D, Mw)).  The
    library streams replica chunks through its stage buffers (the running join kept in HBM, the
    deferred removes settled once against the final clock); the reference's left fold for any
    input states (include/crdt_gpu.h)."""
    ctx = ctx or HostContext.default()
    c = clock[None] if clock.ndim == 2 else clock
    e = entries[None] if entries.ndim == 3 else entries
    c = np.ascontiguousarray(_u64(c, "clock"))
    e = np.ascontiguousarray(_u64(e, "entries"))
    G, R, A = c.shape
    M = e.shape[2]
    Mw = (M + 63) // 64
    b = _abi.OrswotBatch()
    b.G, b.R, b.M, b.A = G, R, M, A
    b.clock, b.clock_rstride, b.clock_gstride = c.ctypes.data, A, R * A
    b.entries, b.entry_mstride, b.entry_rstride, b.entry_gstride = e.ctypes.data, A, M * A, R * M * A
    D = 0
    keep_alive = []
    if def_off is not None:
        off = (ctypes.c_size_t * (G + 1))(*[int(x) for x in def_off])
        keep_alive.append(off)
        b.def_off = off
        D = int(def_off[-1])
        dcl = np.ascontiguousarray(_u64(def_clock, "def_clock"))
        dmb = np.ascontiguousarray(_u64(def_members, "def_members"))
        keep_alive += [dcl, dmb]
        b.def_clock, b.def_members = dcl.ctypes.data, dmb.ctypes.data
    out = OrswotHostLub(np.zeros((G, A), np.uint64), np.zeros((G, M, A), np.uint64), np.zeros(D, np.uint8),
                        np.zeros((D, Mw), np.uint64))
    o = _abi.OrswotOut()
    o.clock, o.entries = out.clock.ctypes.data, out.entries.ctypes.data
    o.def_keep = out.def_keep.ctypes.data if D else None
    o.def_members = out.def_members.ctypes.data if D else None
    ctx.call("crdt_orswot_lub_many", ctypes.byref(b), ctypes.byref(o))
    if clock.ndim == 2:
        return OrswotHostLub(out.clock[0], out.entries[0], out.def_keep, out.def_members)
    return out


def orswot_merge_batch(self_states, other_states, ctx: Optional[HostContext] = None) -> np.ndarray:
    """crdt_orswot_merge_batch on host arrays, in place on self: each side a tuple (clock (N, A),
    entries (N, M, A), def_clock (N, Dcap, A), def_members (N, Dcap, Mw), def_count (N,) uint32)
    of C-contiguous arrays.  Returns status (N,) uint32."""
    ctx = ctx or HostContext.default()
    structs = []
    for side in (self_states, other_states):
        clock, entries, dcl, dmb, cnt = side
        for a in (clock, entries, dcl, dmb, cnt):
            if not a.flags.c_contiguous:
                raise ValueError("orswot_merge_batch: C-contiguous arrays required")
        N, A = clock.shape
        M = entries.shape[1]
        st = _abi.OrswotStates()
        st.N, st.M, st.A, st.Dcap = N, M, A, dcl.shape[1]
        st.clock, st.clock_stride = clock.ctypes.data, A
        st.entries, st.entry_mstride, st.entry_sstride = entries.ctypes.data, A, M * A
        st.def_clock, st.def_members, st.def_count = dcl.ctypes.data, dmb.ctypes.data, cnt.ctypes.data
        structs.append(st)
    status = np.zeros(self_states[0].shape[0], np.uint32)
    ctx.call("crdt_orswot_merge_batch", ctypes.byref(structs[0]), ctypes.byref(structs[1]), _ptr(status))
    return status


class MapHostLub(NamedTuple):
    clock: np.ndarray     # (G, A)
    ec: np.ndarray        # (G, K, A)
    vclk: np.ndarray      # (G, K, Vout, A)
    vval: np.ndarray      # (G, K, Vout)
    nval: np.ndarray      # (G, K) uint32
    flags: np.ndarray     # (G,) uint32
    def_keep: np.ndarray  # (D,) uint8
    def_keys: np.ndarray  # (D, Kw)


def map_lub_many(clock, ec, vclk, vval, def_off=None, def_row=None, def_clock=None, def_keys=None, vout: int = 4,
                 ctx: Optional[HostContext] = None) -> MapHostLub:
    """crdt_map_lub_many on host arrays (one group): clock (R, A), ec (R, K, A), vclk (R, K, V, A),
    vval (R, K, V); removes pooled (def_off [0, D], def_row (D,) uint32, def_clock (D, A),
    def_keys (D, Kw)).  The library streams replica chunks through its stage buffers, the running
    fold carried as replica 0 of the next chunk (exact for any input: the fold is the exact left
    fold); a key needing more than 8 value slots mid-fold falls back to whole-batch staging."""
    ctx = ctx or HostContext.default()
    arrs = [np.ascontiguousarray(_u64(x, n)) for x, n in ((clock, "clock"), (ec, "ec"), (vclk, "vclk"), (vval, "vval"))]
    c, e, vc, vv = arrs
    R, A = c.shape
    K, V = e.shape[1], vc.shape[2]
    Kw = (K + 63) // 64
    b = _abi.MapBatch()
    b.G, b.R, b.K, b.A, b.V = 1, R, K, A, V
    b.clock, b.clock_rstride, b.clock_gstride = c.ctypes.data, A, R * A
    b.ec, b.ec_rstride, b.ec_gstride = e.ctypes.data, K * A, R * K * A
    b.vclk, b.vclk_rstride, b.vclk_gstride = vc.ctypes.data, K * V * A, R * K * V * A
    b.vval, b.vval_rstride, b.vval_gstride = vv.ctypes.data, K * V, R * K * V
    D = 0
    keep = [arrs]
    if def_off is not None and int(def_off[-1]):
        D = int(def_off[-1])
        off = (ctypes.c_size_t * 2)(0, D)
        dr = np.ascontiguousarray(def_row, dtype=np.uint32)
        dcl = np.ascontiguousarray(_u64(def_clock, "def_clock"))
        dks = np.ascontiguousarray(_u64(def_keys, "def_keys"))
        keep += [off, dr, dcl, dks]
        b.def_off, b.def_row, b.def_clock, b.def_keys = off, dr.ctypes.data, dcl.ctypes.data, dks.ctypes.data
    out = MapHostLub(np.zeros((1, A), np.uint64), np.zeros((1, K, A), np.uint64), np.zeros((1, K, vout, A), np.uint64),
                     np.zeros((1, K, vout), np.uint64), np.zeros((1, K), np.uint32), np.zeros(1, np.uint32),
                     np.zeros(D, np.uint8), np.zeros((D, Kw), np.uint64))
    o = _abi.MapOut()
    o.Vout, o.Vstate = vout, 0
    o.clock, o.ec, o.vclk, o.vval = (x.ctypes.data for x in (out.clock, out.ec, out.vclk, out.vval))
    o.nval, o.flags = out.nval.ctypes.data, out.flags.ctypes.data
    o.def_keep = out.def_keep.ctypes.data if D else None
    o.def_keys = out.def_keys.ctypes.data if D else None
    ctx.call("crdt_map_lub_many", ctypes.byref(b), ctypes.byref(o))
    return out


def map_merge_batch(self_states, other_states, ctx: Optional[HostContext] = None) -> np.ndarray:
    """crdt_map_merge_batch on host arrays, in place on self: each side a tuple (clock (N, A),
    ec (N, K, A), vclk (N, K, V, A), vval (N, K, V), def_clock (N, Dcap, A), def_keys (N, Dcap, Kw),
    def_count (N,) uint32) of C-contiguous arrays.  Returns status (N,) uint32."""
    ctx = ctx or HostContext.default()
    ss, dd = [], []
    for side in (self_states, other_states):
        clock, ec, vclk, vval, dcl, dks, cnt = side
        for a in side:
            if not a.flags.c_contiguous:
                raise ValueError("map_merge_batch: C-contiguous arrays required")
        N, A = clock.shape
        K, V = ec.shape[1], vclk.shape[2]
        s = _abi.MapStates()
        s.N, s.K, s.A, s.V = N, K, A, V
        s.clock, s.clock_stride, s.ec, s.ec_stride = clock.ctypes.data, A, ec.ctypes.data, K * A
        s.vclk, s.vclk_stride, s.vval, s.vval_stride = vclk.ctypes.data, K * V * A, vval.ctypes.data, K * V
        d = _abi.MapDeferred()
        d.clock, d.keys, d.count, d.Dcap = dcl.ctypes.data, dks.ctypes.data, cnt.ctypes.data, dcl.shape[1]
        ss.append(s)
        dd.append(d)
    status = np.zeros(self_states[0].shape[0], np.uint32)
    ctx.call("crdt_map_merge_batch", ctypes.byref(ss[0]), ctypes.byref(dd[0]), ctypes.byref(ss[1]),
             ctypes.byref(dd[1]), _ptr(status))
    return status


# ---- the value-typed Maps (round 5): whole-batch staging in the library ----------------------------
def _def_pool(b, def_off, def_row, def_clock, def_keys, keep):
    D = 0
    if def_off is not None and int(def_off[-1]):
        D = int(def_off[-1])
        off = (ctypes.c_size_t * 2)(0, D)
        dr = np.ascontiguousarray(def_row, dtype=np.uint32)
        dcl = np.ascontiguousarray(_u64(def_clock, "def_clock"))
        dks = np.ascontiguousarray(_u64(def_keys, "def_keys"))
        keep += [off, dr, dcl, dks]
        b.def_off, b.def_row, b.def_clock, b.def_keys = off, dr.ctypes.data, dcl.ctypes.data, dks.ctypes.data
    return D


def map_counter_lub_many(clock, ec, val, def_off=None, def_row=None, def_clock=None, def_keys=None,
                         ctx: Optional[HostContext] = None) -> dict:
    """crdt_map_counter_lub_many on host arrays (one group): clock (R, A), ec (R, K, A), val (R, K, W, A)
    (W = 1 GCounter, 2 PNCounter P | N); the Map's removes pooled as for map_lub_many."""
    ctx = ctx or HostContext.default()
    c, e, v = (np.ascontiguousarray(_u64(x, n)) for x, n in ((clock, "clock"), (ec, "ec"), (val, "val")))
    R, A = c.shape
    K, W = e.shape[1], v.shape[2]
    b = _abi.MapCounterBatch()
    b.G, b.R, b.K, b.A, b.W = 1, R, K, A, W
    b.clock, b.clock_rstride, b.clock_gstride = c.ctypes.data, A, R * A
    b.ec, b.ec_rstride, b.ec_gstride = e.ctypes.data, K * A, R * K * A
    b.val, b.val_rstride, b.val_gstride = v.ctypes.data, K * W * A, R * K * W * A
    keep = [c, e, v]
    D = _def_pool(b, def_off, def_row, def_clock, def_keys, keep)
    Kw = (K + 63) // 64
    out = dict(clock=np.zeros((1, A), np.uint64), ec=np.zeros((1, K, A), np.uint64),
               val=np.zeros((1, K, W, A), np.uint64), flags=np.zeros(1, np.uint32), def_keep=np.zeros(D, np.uint8),
               def_keys=np.zeros((D, Kw), np.uint64))
    o = _abi.MapCounterOut()
    o.clock, o.ec, o.val, o.flags = (out[n].ctypes.data for n in ("clock", "ec", "val", "flags"))
    o.def_keep = out["def_keep"].ctypes.data if D else None
    o.def_keys = out["def_keys"].ctypes.data if D else None
    ctx.call("crdt_map_counter_lub_many", ctypes.byref(b), ctypes.byref(o))
    return out


def map_orswot_lub_many(clock, ec, oc, ent, vd_off, vd_clock=None, vd_mem=None, def_off=None, def_row=None,
                        def_clock=None, def_keys=None, ctx: Optional[HostContext] = None, vd_cap: int = 16) -> dict:
    """crdt_map_orswot_lub_many on host arrays (one group): clock (R, A), ec / oc (R, K, A), ent (R, K, M, A),
    the nested removes as a CSR over (r, k): vd_off (R*K + 1,), vd_clock (Dv, A), vd_mem (Dv,) ((Dv, Mw)
    member-mask words past M = 64; the results' vd_mem then (1, K, Vd, Mw)); vd_cap = Vd nested slots
    per key in the result (>= 16)."""
    ctx = ctx or HostContext.default()
    c, e, o_, m = (np.ascontiguousarray(_u64(x, n)) for x, n in ((clock, "clock"), (ec, "ec"), (oc, "oc"), (ent, "ent")))
    R, A = c.shape
    K, M = e.shape[1], m.shape[2]
    vo = np.ascontiguousarray(_u64(vd_off, "vd_off")) if vd_off is not None else None  # (None: R == 0 only)
    Dv = int(vd_clock.shape[0]) if vd_clock is not None else 0
    vc = np.ascontiguousarray(_u64(vd_clock, "vd_clock")) if Dv else None
    vm = np.ascontiguousarray(_u64(vd_mem, "vd_mem")) if Dv else None
    b = _abi.MapOrswotBatch()
    b.G, b.R, b.K, b.M, b.A = 1, R, K, M, A
    b.clock, b.ec, b.oc, b.ent = (x.ctypes.data for x in (c, e, o_, m))
    b.vd_off, b.Dv = (vo.ctypes.data if vo is not None else None), Dv
    if Dv:
        b.vd_clock, b.vd_mem = vc.ctypes.data, vm.ctypes.data
    keep = [c, e, o_, m, vo, vc, vm]
    D = _def_pool(b, def_off, def_row, def_clock, def_keys, keep)
    Kw = (K + 63) // 64
    out = dict(clock=np.zeros((1, A), np.uint64), ec=np.zeros((1, K, A), np.uint64), oc=np.zeros((1, K, A), np.uint64),
               ent=np.zeros((1, K, M, A), np.uint64), vd_n=np.zeros((1, K), np.uint32),
               vd_clock=np.zeros((1, K, vd_cap, A), np.uint64),
               vd_mem=np.zeros((1, K, vd_cap) if M <= 64 else (1, K, vd_cap, (M + 63) // 64), np.uint64),
               flags=np.zeros(1, np.uint32), def_keep=np.zeros(D, np.uint8), def_keys=np.zeros((D, Kw), np.uint64))
    ob = _abi.MapOrswotOut()
    for n in ("clock", "ec", "oc", "ent", "vd_n", "vd_clock", "vd_mem", "flags"):
        setattr(ob, n, out[n].ctypes.data)
    ob.def_keep = out["def_keep"].ctypes.data if D else None
    ob.def_keys = out["def_keys"].ctypes.data if D else None
    ob.Vd = vd_cap
    ctx.call("crdt_map_orswot_lub_many", ctypes.byref(b), ctypes.byref(ob))
    return out


def map_nested_lub_many(clock, ec, ic, iec, ivc, ivv, id_off, id_clock=None, id_keys=None, def_off=None, def_row=None,
                        def_clock=None, def_keys=None, ctx: Optional[HostContext] = None, id_cap: int = 16,
                        v_cap: int = 8) -> dict:
    """crdt_map_nested_lub_many on host arrays (one group): clock (R, A), ec / ic (R, K, A), iec (R, K, K2, A),
    ivc (R, K, K2, V, A), ivv (R, K, K2, V), the inner removes as a CSR over (r, k) (id_keys (Di,), or
    (Di, K2w) mask words past K2 = 64, as the results' id_keys (1, K, Id[, K2w])); id_cap = Id inner
    slots per key in the result (>= 16)."""
    ctx = ctx or HostContext.default()
    arrs = [np.ascontiguousarray(_u64(x, n)) for x, n in ((clock, "clock"), (ec, "ec"), (ic, "ic"), (iec, "iec"),
                                                          (ivc, "ivc"), (ivv, "ivv"))]
    c, e, i_, ie, vc, vv = arrs
    io = np.ascontiguousarray(_u64(id_off, "id_off")) if id_off is not None else None  # (None: R == 0 only)
    R, A = c.shape
    K, K2, V = e.shape[1], ie.shape[2], vc.shape[3]
    Di = int(id_clock.shape[0]) if id_clock is not None else 0
    idc = np.ascontiguousarray(_u64(id_clock, "id_clock")) if Di else None
    idk = np.ascontiguousarray(_u64(id_keys, "id_keys")) if Di else None
    b = _abi.MapNestedBatch()
    b.G, b.R, b.K, b.K2, b.V, b.A = 1, R, K, K2, V, A
    b.clock, b.ec, b.ic, b.iec, b.ivc, b.ivv = (x.ctypes.data for x in (c, e, i_, ie, vc, vv))
    b.id_off, b.Di = (io.ctypes.data if io is not None else None), Di
    if Di:
        b.id_clock, b.id_keys = idc.ctypes.data, idk.ctypes.data
    keep = arrs + [io, idc, idk]
    D = _def_pool(b, def_off, def_row, def_clock, def_keys, keep)
    Kw = (K + 63) // 64
    out = dict(clock=np.zeros((1, A), np.uint64), ec=np.zeros((1, K, A), np.uint64), ic=np.zeros((1, K, A), np.uint64),
               iec=np.zeros((1, K, K2, A), np.uint64), ivc=np.zeros((1, K, K2, v_cap, A), np.uint64),
               ivv=np.zeros((1, K, K2, v_cap), np.uint64), nval=np.zeros((1, K, K2), np.uint32),
               id_n=np.zeros((1, K), np.uint32), id_clock=np.zeros((1, K, id_cap, A), np.uint64),
               id_keys=np.zeros((1, K, id_cap) if K2 <= 64 else (1, K, id_cap, (K2 + 63) // 64), np.uint64),
               flags=np.zeros(1, np.uint32), def_keep=np.zeros(D, np.uint8),
               def_keys=np.zeros((D, Kw), np.uint64))
    ob = _abi.MapNestedOut()
    for n in ("clock", "ec", "ic", "iec", "ivc", "ivv", "nval", "id_n", "id_clock", "id_keys", "flags"):
        setattr(ob, n, out[n].ctypes.data)
    ob.def_keep = out["def_keep"].ctypes.data if D else None
    ob.def_keys = out["def_keys"].ctypes.data if D else None
    ob.Id, ob.Vs = id_cap, v_cap
    ctx.call("crdt_map_nested_lub_many", ctypes.byref(b), ctypes.byref(ob))
    return out
