"""Device context: one libcrdt_gpu ctx per (process, device), launching on torch's stream."""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import torch

from . import _abi

U64_DTYPES = (torch.int64, torch.uint64)


class Context:
    """Owns a `crdt_ctx` bound to one HIP device (include/crdt_gpu.h: crdt_ctx_create).

    Every call is issued on torch's *current* stream for the device, so results are ordered
    with the torch ops around them.  Device tensors are torch int64 (or uint64) tensors
    holding the u64 bit patterns of the reference's `u64` counters/markers.
    """

    _by_device: Dict[int, "Context"] = {}

    def __init__(self, device: int = 0):
        self.lib = _abi.load()
        if not torch.cuda.is_available():
            raise _abi.CrdtGpuUnavailable("no HIP device visible to torch: libcrdt_gpu needs an MI355X")
        self.device = int(device)
        ptr = ctypes.c_void_p()
        rc = self.lib.crdt_ctx_create(self.device, ctypes.byref(ptr))
        _abi.check(None, "crdt_ctx_create", rc)
        self.ptr = ptr

    @classmethod
    def default(cls, device: Optional[int] = None) -> "Context":
        if device is None:
            device = torch.cuda.current_device()
        ctx = cls._by_device.get(device)
        if ctx is None:
            ctx = cls(device)
            cls._by_device[device] = ctx
        return ctx

    def close(self) -> None:
        if getattr(self, "ptr", None):
            self.lib.crdt_ctx_destroy(self.ptr)
            self.ptr = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    # -- plumbing -------------------------------------------------------------------------
    def bind_stream(self) -> None:
        s = torch.cuda.current_stream(self.device).cuda_stream
        _abi.check(self.ptr, "crdt_ctx_set_stream", self.lib.crdt_ctx_set_stream(self.ptr, ctypes.c_void_p(s)))

    def call(self, name: str, *args) -> None:
        self.bind_stream()
        rc = getattr(self.lib, name)(self.ptr, *args)
        _abi.check(self.ptr, name, rc)

    def synchronize(self) -> None:
        self.call("crdt_ctx_synchronize")

    def set_timing(self, enable: bool) -> None:
        self.call("crdt_ctx_set_timing", 1 if enable else 0)

    def timing(self, name: str) -> Tuple[float, int]:
        ms = ctypes.c_double()
        n = ctypes.c_uint64()
        self.call("crdt_ctx_timing", name.encode(), ctypes.byref(ms), ctypes.byref(n))
        return ms.value, n.value

    def timing_reset(self) -> None:
        self.call("crdt_ctx_timing_reset")

    def tune(self, spec: str) -> None:
        """Override launch-geometry knobs ("key=value,...", CRDT_TUNE syntax); never changes results."""
        self.call("crdt_ctx_tune", spec.encode())

    def device_empty(self, shape, dtype: torch.dtype = torch.int64) -> Optional[torch.Tensor]:
        """An uninitialised tensor on this ctx's GPU in one physically contiguous block
        (crdt_device_alloc), freed when the last view of it dies; None when no such block is free
        (the caller then takes any device memory, e.g. torch.empty)."""
        n = 1
        for x in shape:
            n *= int(x)
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        p = ctypes.c_void_p()
        rc = self.lib.crdt_device_alloc(self.ptr, max(nbytes, 1), ctypes.byref(p))
        if rc != 0 or not p.value:
            return None
        typestr = {torch.int64: "<i8", torch.int32: "<i4", torch.uint8: "|u1", torch.int8: "|i1"}[dtype]
        blk = _DeviceBlock(self.lib, p.value, tuple(int(x) for x in shape), typestr)
        return torch.as_tensor(blk, device=torch.device("cuda", self.device))

    # -- tensor checks ----------------------------------------------------------------------
    def check_tensor(self, t: torch.Tensor, what: str, dtypes=None) -> None:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{what}: expected a torch.Tensor")
        if dtypes is not None:
            if t.dtype not in dtypes:
                raise TypeError(f"{what}: dtype {t.dtype}; expected one of {dtypes}")
        elif t.dtype not in U64_DTYPES:
            raise TypeError(f"{what}: dtype {t.dtype}; expected int64/uint64 holding u64 bits")
        if t.device.type != "cuda" or t.device.index != self.device:
            raise ValueError(f"{what}: tensor on {t.device}; expected cuda:{self.device}")


class _DeviceBlock:
    """A crdt_device_alloc block seen by torch through __cuda_array_interface__; torch holds a
    reference for as long as a tensor views it, and the block is freed after the last one."""

    def __init__(self, lib, ptr: int, shape, typestr: str):
        self._lib, self._ptr = lib, ptr
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False),
                                         "version": 2, "strides": None}

    def __del__(self):
        if self._ptr:
            self._lib.crdt_device_free(None, ctypes.c_void_p(self._ptr))
            self._ptr = 0


def dptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def synth_fill(ctx: Context, out: torch.Tensor, seed: int, kind: int, first_row: int = 0) -> torch.Tensor:
    """Fill a (rows, width) tensor with rows [first_row, first_row+rows) of the counter-based
    synthetic matrix, generated in HBM (crdt_synth_fill)."""
    ctx.check_tensor(out, "synth_fill.out")
    if out.dim() == 1:
        rows, width, rs = 1, out.shape[0], out.shape[0]
    else:
        o2 = out.reshape(-1, out.shape[-1]) if out.is_contiguous() else out
        if o2.dim() != 2 or o2.stride(1) != 1:
            raise ValueError("synth_fill: need a row-contiguous 2-D view")
        rows, width, rs = o2.shape[0], o2.shape[1], o2.stride(0)
    ctx.call("crdt_synth_fill", dptr(out), rows, width, rs, int(first_row), ctypes.c_uint64(seed & (2**64 - 1)), int(kind))
    return out
