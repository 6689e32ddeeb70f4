"""Replica-sharded lub through the C ABI's own RCCL communicator (include/crdt_gpu.h,
"multi-GPU"): the path a Rust caller takes, with no torch.distributed in the exchange.

    uid = unique_id()                       # rank 0; distribute the 128 bytes to every rank
    comm_init(ctx, uid, nranks, rank)       # collective
    # or the caller's own collectives instead of RCCL (crdt_ctx_comm_init_ops), e.g. gloo:
    comm_init_ops(ctx, TorchCommOps(), nranks, rank)
    lub_many_sharded("gcounter", shard)     # collective: every rank gets the global lub
    orswot_lub_many_sharded(clock, entries, def_off, def_clock, def_members)
    lwwreg_lub_many_sharded(marker, val, base)       # replicas [base, base + R_k) of the global order
    map_lub_many_sharded(clock, ec, vclk, vval, k0, K, ...)   # KEY shards [k0, k0 + K_k)

Every *_sharded call is collective and agrees on its validation status first: a bad argument on one
rank makes EVERY rank raise (CrdtGpuError), none blocks.  `crdts_gpu.dist` is the torch.distributed
twin of the same exchange (gloo-testable on CPU)."""
from __future__ import annotations

import ctypes
from typing import NamedTuple, Optional, Sequence

import numpy as np
import torch

from . import _abi
from ._lattice import _geometry
from .context import Context, dptr


def unique_id() -> bytes:
    lib = _abi.load()
    buf = (ctypes.c_uint8 * _abi.CRDT_UNIQUE_ID_BYTES)()
    _abi.check(None, "crdt_comm_unique_id", lib.crdt_comm_unique_id(buf))
    return bytes(buf)


def comm_init(ctx: Context, uid: bytes, nranks: int, rank: int) -> None:
    if len(uid) != _abi.CRDT_UNIQUE_ID_BYTES:
        raise ValueError(f"comm_init: unique id must be {_abi.CRDT_UNIQUE_ID_BYTES} bytes")
    buf = (ctypes.c_uint8 * _abi.CRDT_UNIQUE_ID_BYTES).from_buffer_copy(uid)
    ctx.call("crdt_ctx_comm_init", buf, int(nranks), int(rank))


def comm_note(ctx: Context):
    """(which RCCL the communicator runs on, its version code, the rccl.h version of the types) —
    crdt_ctx_comm_note.  One RCCL per process: inside a torch process the library binds torch's."""
    rt, hd = ctypes.c_int(), ctypes.c_int()
    txt = _abi.load().crdt_ctx_comm_note(ctx.ptr, ctypes.byref(rt), ctypes.byref(hd))
    return (txt or b"").decode(), rt.value, hd.value


class TorchCommOps:
    """crdt_comm_ops backed by torch.distributed on host tensors (gloo, or any backend with CPU
    collectives): the caller's-own-transport seam of the C ABI.  The unsigned reductions are done
    exactly on uint64 after an all-gather (gloo's int64 MAX / MIN are signed)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.errors = []

        def allgather(user, send, recv, nbytes):
            try:
                src = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(send))
                t = torch.from_numpy(src.copy())
                parts = [torch.empty_like(t) for _ in range(self.world)]
                self.dist.all_gather(parts, t, group=self.group)
                dst = np.ctypeslib.as_array((ctypes.c_uint8 * (nbytes * self.world)).from_address(recv))
                dst[:] = torch.cat(parts).numpy()
                return 0
            except Exception as e:  # noqa: BLE001 - reported to the C side as a failed collective
                self.errors.append(repr(e))
                return 1

        def allreduce(user, buf, n, op):
            try:
                arr = np.ctypeslib.as_array(buf, shape=(n,))
                t = torch.from_numpy(arr.view(np.int64).copy())
                parts = [torch.empty_like(t) for _ in range(self.world)]
                self.dist.all_gather(parts, t, group=self.group)
                st = np.stack([p.numpy().view(np.uint64) for p in parts])
                if op == _abi.CRDT_RED_MAX:
                    arr[:] = st.max(0)
                elif op == _abi.CRDT_RED_MIN:
                    arr[:] = st.min(0)
                elif op == _abi.CRDT_RED_SUM:
                    arr[:] = st.sum(0, dtype=np.uint64)
                else:
                    return 2
                return 0
            except Exception as e:  # noqa: BLE001
                self.errors.append(repr(e))
                return 1

        self._ag = _abi.ALLGATHER_FN(allgather)
        self._ar = _abi.ALLREDUCE_FN(allreduce)
        self.ops = _abi.CommOps(None, self._ag, self._ar)


def comm_init_ops(ctx: Context, ops, nranks: int, rank: int) -> None:
    """crdt_ctx_comm_init_ops: the sharded entry points exchange through `ops` (an object with a
    `.ops` crdt_comm_ops struct, e.g. TorchCommOps) instead of RCCL.  The ctx keeps a reference."""
    ctx.call("crdt_ctx_comm_init_ops", ctypes.byref(ops.ops), int(nranks), int(rank))
    ctx._comm_ops = ops  # the callbacks must outlive the communicator


def comm_destroy(ctx: Context) -> None:
    ctx.call("crdt_ctx_comm_destroy")
    ctx._comm_ops = None


def comm_info(ctx: Context):
    n, r = ctypes.c_int(), ctypes.c_int()
    ctx.call("crdt_ctx_comm_info", ctypes.byref(n), ctypes.byref(r))
    return n.value, r.value


_WIDTH_DIV = {"vclock": 1, "gcounter": 1, "pncounter": 2, "gset": 1}


def lub_many_sharded(kind: str, shard: torch.Tensor, ctx: Optional[Context] = None) -> torch.Tensor:
    """Global lub of the replicas held across the ctx's ranks; `shard` is this rank's (R_k, W)
    or (G, R_k, W) block.  Returns (W,) or (G, W), identical on every rank."""
    if kind not in _WIDTH_DIV:
        raise ValueError(f"lub_many_sharded: unknown kind {kind}")
    ctx = ctx or Context.default(shard.device.index)
    ctx.check_tensor(shard, f"{kind}.lub_many_sharded")
    G, R, W, rstride, gstride = _geometry(shard, f"{kind}.lub_many_sharded")
    if W % _WIDTH_DIV[kind]:
        raise ValueError(f"{kind}.lub_many_sharded: row width {W} not a multiple of {_WIDTH_DIV[kind]}")
    out = torch.empty((G, W), dtype=shard.dtype, device=shard.device)
    ctx.call(f"crdt_{kind}_lub_many_sharded", dptr(shard), G, R, W // _WIDTH_DIV[kind], rstride, gstride, dptr(out))
    return out[0] if shard.dim() == 2 else out


def lub_many_multi_sharded(items, ctx: Optional[Context] = None):
    """crdt_lub_many_multi_sharded: items (kind, shard, out) as _lattice.lub_many_multi, each out
    the global lub over the ranks (one fused local launch + one grouped RCCL all-reduce)."""
    from ._lattice import segments
    if not items:
        return []
    ctx = ctx or Context.default(items[0][1].device.index)
    arr = segments(items, ctx)
    ctx.call("crdt_lub_many_multi_sharded", arr, len(items))
    return [o for _, _, o in items]


class OrswotSharded(NamedTuple):
    clock: torch.Tensor        # (G, A)
    entries: torch.Tensor      # (G, M, A)
    def_clock: torch.Tensor    # (ndef, A)   surviving deferred removes
    def_members: torch.Tensor  # (ndef, Mw)  member union per surviving rm clock
    def_group: torch.Tensor    # (ndef,) int32


def orswot_lub_many_sharded(clock: torch.Tensor, entries: torch.Tensor, def_off: Optional[Sequence[int]] = None,
                            def_clock: Optional[torch.Tensor] = None, def_members: Optional[torch.Tensor] = None,
                            ctx: Optional[Context] = None, def_cap: Optional[int] = None) -> OrswotSharded:
    """Rank k's shard: clock (G, R_k, A), entries (G, R_k, M, A) and its deferred removes pooled
    per group (def_off of G+1 entries: a host sequence, or a contiguous int64 cuda tensor —
    crdt_orswot_lub_many_sharded_doff, D_k = def_clock.shape[0] —, def_clock (D_k, A),
    def_members (D_k, Mw))."""
    ctx = ctx or Context.default(clock.device.index)
    ctx.check_tensor(clock, "orswot.lub_many_sharded(clock)")
    ctx.check_tensor(entries, "orswot.lub_many_sharded(entries)")
    if clock.dim() != 3 or entries.dim() != 4 or clock.stride(2) != 1 or entries.stride(3) != 1:
        raise ValueError("orswot.lub_many_sharded: clock (G,R,A) / entries (G,R,M,A), actor axis contiguous")
    G, R, A = clock.shape
    M = entries.shape[2]
    Mw = (M + 63) // 64
    b = _abi.OrswotBatch()
    b.G, b.R, b.M, b.A = G, R, M, A
    b.clock, b.clock_rstride, b.clock_gstride = clock.data_ptr(), clock.stride(1), clock.stride(0)
    b.entries = entries.data_ptr()
    b.entry_mstride, b.entry_rstride, b.entry_gstride = entries.stride(2), entries.stride(1), entries.stride(0)
    off_arr = None
    D = 0
    dev_off = isinstance(def_off, torch.Tensor) and def_off.device.type == "cuda"
    if dev_off:
        if (def_off.dtype not in (torch.int64, torch.uint64) or tuple(def_off.shape) != (G + 1,)
                or not def_off.is_contiguous() or def_off.device.index != ctx.device):
            raise ValueError(f"orswot.lub_many_sharded: a device def_off must be a contiguous ({G + 1},) int64 "
                             f"cuda:{ctx.device} tensor")
        D = 0 if def_clock is None else int(def_clock.shape[0])
        if D:
            for t, nm, w in ((def_clock, "def_clock", A), (def_members, "def_members", Mw)):
                if t is None or not t.is_contiguous() or tuple(t.shape) != (D, w):
                    raise ValueError(f"orswot.lub_many_sharded: {nm} must be a contiguous ({D}, {w}) tensor")
                ctx.check_tensor(t, f"orswot.lub_many_sharded({nm})")
            b.def_clock, b.def_members = def_clock.data_ptr(), def_members.data_ptr()
    elif def_off is not None:
        off = [int(x) for x in def_off]
        if len(off) != G + 1:
            raise ValueError(f"orswot.lub_many_sharded: def_off must have G+1 = {G + 1} entries")
        D = off[-1]
        if D:
            for t, nm, w in ((def_clock, "def_clock", A), (def_members, "def_members", Mw)):
                if t is None or not t.is_contiguous() or tuple(t.shape) != (D, w):
                    raise ValueError(f"orswot.lub_many_sharded: {nm} must be a contiguous ({D}, {w}) tensor")
                ctx.check_tensor(t, f"orswot.lub_many_sharded({nm})")
            b.def_clock, b.def_members = def_clock.data_ptr(), def_members.data_ptr()
        off_arr = (ctypes.c_size_t * (G + 1))(*off)
        b.def_off = ctypes.cast(off_arr, ctypes.POINTER(ctypes.c_size_t))
    cap = def_cap if def_cap is not None else max(1, 4 * D + 64)
    oc = torch.empty((G, A), dtype=clock.dtype, device=clock.device)
    oe = torch.empty((G, M, A), dtype=clock.dtype, device=clock.device)
    odc = torch.empty((cap, A), dtype=clock.dtype, device=clock.device)
    odm = torch.empty((cap, Mw), dtype=clock.dtype, device=clock.device)
    odg = torch.empty((cap,), dtype=torch.int32, device=clock.device)
    nd = ctypes.c_size_t()
    o = _abi.OrswotShardedOut()
    o.clock, o.entries, o.def_cap = oc.data_ptr(), oe.data_ptr(), cap
    o.def_clock, o.def_members, o.def_group = odc.data_ptr(), odm.data_ptr(), odg.data_ptr()
    o.ndef = ctypes.pointer(nd)
    if dev_off:
        ctx.call("crdt_orswot_lub_many_sharded_doff", ctypes.byref(b), def_off.data_ptr(), D, ctypes.byref(o))
    else:
        ctx.call("crdt_orswot_lub_many_sharded", ctypes.byref(b), ctypes.byref(o))
    n = nd.value
    if n > cap:  # more survivors than room: run again with exactly enough
        return orswot_lub_many_sharded(clock, entries, def_off, def_clock, def_members, ctx, def_cap=n)
    return OrswotSharded(oc, oe, odc[:n], odm[:n], odg[:n])


def deferred_groups(res: OrswotSharded, G: int):
    """Egress: per group, {(rm clock tuple, frozenset of members)} of the surviving removes."""
    out = [set() for _ in range(G)]
    dc = res.def_clock.cpu().numpy().view(np.uint64)
    dm = res.def_members.cpu().numpy().view(np.uint64)
    for d, g in enumerate(res.def_group.cpu().numpy().tolist()):
        ms = []
        for w, x in enumerate(dm[d].tolist()):
            while x:
                ms.append(w * 64 + (x & -x).bit_length() - 1)
                x &= x - 1
        out[g].add((tuple(int(v) for v in dc[d]), frozenset(ms)))
    return out


def lwwreg_lub_many_sharded(marker: torch.Tensor, val: torch.Tensor, base: int, ctx: Optional[Context] = None):
    """LWWReg fold over replicas split in rank order (crdt_lwwreg_lub_many_sharded): rank k passes its
    (R_k,) or (G, R_k) marker / val block and the global index `base` of its first replica.  Returns
    (marker, val, first_conflict) of the GLOBAL left fold on every rank (first_conflict -1 = none)."""
    ctx = ctx or Context.default(marker.device.index)
    ctx.check_tensor(marker, "lwwreg.lub_many_sharded(marker)")
    ctx.check_tensor(val, "lwwreg.lub_many_sharded(val)")
    if marker.shape != val.shape or marker.dim() not in (1, 2):
        raise ValueError("lwwreg.lub_many_sharded: marker and val must share a (R,) or (G, R) shape")
    squeeze = marker.dim() == 1
    m2 = marker.reshape(1, -1) if squeeze else marker
    v2 = val.reshape(1, -1) if squeeze else val
    G, R = m2.shape
    if R and (m2.stride(1) != 1 or v2.stride(1) != 1 or m2.stride(0) != v2.stride(0)):
        raise ValueError("lwwreg.lub_many_sharded: rows must be contiguous with equal strides")
    om = torch.empty(G, dtype=torch.int64, device=marker.device)
    ov, fc = torch.empty_like(om), torch.empty_like(om)
    ctx.call("crdt_lwwreg_lub_many_sharded", dptr(m2) if R else None, dptr(v2) if R else None, G, R,
             m2.stride(0) if G > 1 else max(R, 1), ctypes.c_uint64(int(base)), dptr(om), dptr(ov), dptr(fc))
    return (om[0], ov[0], fc[0]) if squeeze else (om, ov, fc)


def map_lub_many_sharded(clock: torch.Tensor, ec: torch.Tensor, vclk: torch.Tensor, vval: torch.Tensor, k0: int,
                         K: int, def_off=None, def_row=None, def_clock=None, def_keys=None, vout: int = 4,
                         ctx: Optional[Context] = None, vstate: int = 0):
    """Key-sharded Map<K, MVReg> fold (crdt_map_lub_many_sharded): this rank's keys [k0, k0 + K_k) of
    every replica (ec (G, R, K_k, A), ...), every replica clock, the whole deferred list with key
    bitmaps over all K keys.  Returns a map.MapLub of the rank's keys whose def_keys span all K.
    `vstate` (the starting fold-state size) is part of the agreed call: it must match on every rank."""
    from . import map as cmap
    return cmap.lub_many(clock, ec, vclk, vval, def_off=def_off, def_row=def_row, def_clock=def_clock,
                         def_keys=def_keys, vout=vout, ctx=ctx, vstate=vstate,
                         _key_shard=(int(k0), int(K)))


def map_counter_lub_many_sharded(clock: torch.Tensor, ec: torch.Tensor, val: torch.Tensor, k0: int, K: int,
                                 def_off=None, def_row=None, def_clock=None, def_keys=None,
                                 ctx: Optional[Context] = None, check: bool = True):
    """Key-sharded Map<K, GCounter / PNCounter> fold (crdt_map_counter_lub_many_sharded, round 5):
    this rank's keys [k0, k0 + K_k) of every replica (ec (G, R, K_k, A), val (G, R, K_k, W, A)), every
    replica clock, the whole deferred list with key bitmaps over all K keys.  Returns a
    map.MapCounterLub of the rank's keys whose def_keys span all K."""
    from . import map as cmap
    return cmap.counter_lub_many(clock, ec, val, def_off=def_off, def_row=def_row, def_clock=def_clock,
                                 def_keys=def_keys, ctx=ctx, check=check, _key_shard=(int(k0), int(K)))


def map_orswot_lub_many_sharded(clock: torch.Tensor, ec: torch.Tensor, oc: torch.Tensor, ent: torch.Tensor,
                                vd_off: torch.Tensor, k0: int, K: int, vd_clock=None, vd_mem=None, def_off=None,
                                def_row=None, def_clock=None, def_keys=None, ctx: Optional[Context] = None,
                                check: bool = True):
    """Key-sharded Map<K, Orswot> fold (crdt_map_orswot_lub_many_sharded, round 5): this rank's keys
    (ec / oc (G, R, K_k, A), ent (G, R, K_k, M, A), the nested removes' CSR over (g, r, its keys)),
    every replica clock, the whole deferred list with key bitmaps over all K keys."""
    from . import map as cmap
    return cmap.orswot_lub_many(clock, ec, oc, ent, vd_off, vd_clock=vd_clock, vd_mem=vd_mem, def_off=def_off,
                                def_row=def_row, def_clock=def_clock, def_keys=def_keys, ctx=ctx, check=check,
                                _key_shard=(int(k0), int(K)))


def map_nested_lub_many_sharded(clock: torch.Tensor, ec: torch.Tensor, ic: torch.Tensor, iec: torch.Tensor,
                                ivc: torch.Tensor, ivv: torch.Tensor, id_off: torch.Tensor, k0: int, K: int,
                                id_clock=None, id_keys=None, def_off=None, def_row=None, def_clock=None,
                                def_keys=None, ctx: Optional[Context] = None, check: bool = True):
    """Key-sharded Map<K, Map<K2, MVReg>> fold (crdt_map_nested_lub_many_sharded, round 5): this rank's
    outer keys of every replica, every replica clock, the whole outer deferred list with key bitmaps
    over all K keys."""
    from . import map as cmap
    return cmap.nested_lub_many(clock, ec, ic, iec, ivc, ivv, id_off, id_clock=id_clock, id_keys=id_keys,
                                def_off=def_off, def_row=def_row, def_clock=def_clock, def_keys=def_keys, ctx=ctx,
                                check=check, _key_shard=(int(k0), int(K)))
