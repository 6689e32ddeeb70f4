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
    ctx = ctx or HostContext()
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
    ctx = ctx or HostContext()
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
    ctx = ctx or HostContext()
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
    ctx = ctx or HostContext()
    arrs = [_u64(a, n) for a, n in ((self_marker, "self_marker"), (self_val, "self_val"),
                                     (other_marker, "other_marker"), (other_val, "other_val"))]
    N = arrs[0].shape[0]
    if any(a.shape != (N,) or a.strides != (8,) for a in arrs):
        raise ValueError("lwwreg_merge_batch: four contiguous (N,) arrays")
    conflict = np.zeros(N, np.uint8)
    ctx.call("crdt_lwwreg_merge_batch", *[_ptr(a) for a in arrs], N, _ptr(conflict))
    return conflict
