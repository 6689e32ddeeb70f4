"""Batched `Map<K, MVReg<u64, A>, A>` merge (reference: src/map.rs:140-220, src/mvreg.rs:112-128).

Dense layout (keys, actors and MVReg values interned to indices / u64 by the caller, see
`intern`):
    clock (R, A)        or (G, R, A)         replica map clocks
    ec    (R, K, A)     or (G, R, K, A)      entry clocks; key absent <=> row all 0
    vclk  (R, K, V, A)  or (G, R, K, V, A)   MVReg value clocks, slots in Vec order (empty <=> 0)
    vval  (R, K, V)     or (G, R, K, V)      MVReg values
    deferred removes pooled per group:
        def_off   host sequence of G+1 offsets (group g owns [def_off[g], def_off[g+1])), or a
                  (G+1,) int64 device tensor (crdt_map_lub_many_doff: D = def_clock.shape[0], no host sync)
        def_row   (D,) device int32: replica index within the group (non-decreasing per group)
        def_clock (D, A) rm clocks; def_keys (D, ceil(K/64)) key bitmaps

lub_many computes, per group, the exact left fold `acc = Map::new(); for r: acc.merge(r)`
(test/map.rs:660-692 merges this way) and returns MapLub(clock (G,A), ec (G,K,A),
vclk (G,K,Vout,A), vval (G,K,Vout), nval (G,K) int32, flags (G,) int32, def_keep, def_keys).
With check=True (default) a flagged group raises: bit 0 = more than `vout` values on a key
(retry with a larger vout), bit 1 = def_row not sorted / out of range (or, for device def_off, the
offsets bounding the group invalid); bit 2 (the fold state
ran out of value slots mid-fold) first reruns the fold with the largest state (8 values).
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple, Optional

import numpy as np
import torch

from . import _abi
from .context import Context


class MapLub(NamedTuple):
    clock: torch.Tensor
    ec: torch.Tensor
    vclk: torch.Tensor
    vval: torch.Tensor
    nval: torch.Tensor
    flags: torch.Tensor
    def_keep: Optional[torch.Tensor]
    def_keys: Optional[torch.Tensor]


class MapCapacityError(RuntimeError):
    """A folded key holds more MVReg values than the output slots (flags bit 0)."""


def lub_many(clock: torch.Tensor, ec: torch.Tensor, vclk: torch.Tensor, vval: torch.Tensor,
             def_off=None, def_row: Optional[torch.Tensor] = None,
             def_clock: Optional[torch.Tensor] = None, def_keys: Optional[torch.Tensor] = None,
             vout: int = 4, ctx: Optional[Context] = None, check: bool = True,
             vstate: int = 0, _key_shard: Optional[tuple] = None) -> MapLub:
    """`_key_shard=(k0, K_total)`: this rank's keys [k0, k0 + K) of a key-sharded fold through the
    C ABI's communicator (crdt_map_lub_many_sharded; use crdts_gpu.shard.map_lub_many_sharded):
    def_keys / the returned def_keys are then over all K_total keys."""
    ctx = ctx or Context.default(clock.device.index)
    for t, nm in ((clock, "clock"), (ec, "ec"), (vclk, "vclk"), (vval, "vval")):
        ctx.check_tensor(t, f"map.lub_many({nm})")
    squeeze = clock.dim() == 2
    c = clock.unsqueeze(0) if squeeze else clock
    e = ec.unsqueeze(0) if squeeze else ec
    vc = vclk.unsqueeze(0) if squeeze else vclk
    vv = vval.unsqueeze(0) if squeeze else vval
    if c.dim() != 3 or e.dim() != 4 or vc.dim() != 5 or vv.dim() != 4:
        raise ValueError("map.lub_many: clock (G,R,A), ec (G,R,K,A), vclk (G,R,K,V,A), vval (G,R,K,V) expected")
    G, R, A = c.shape
    K, V = e.shape[2], vc.shape[3]
    if (tuple(e.shape) != (G, R, K, A) or tuple(vc.shape) != (G, R, K, V, A)
            or tuple(vv.shape) != (G, R, K, V)):
        raise ValueError(f"map.lub_many: shapes clock {tuple(c.shape)} ec {tuple(e.shape)} "
                         f"vclk {tuple(vc.shape)} vval {tuple(vv.shape)} do not agree")
    # per-replica blocks must be packed (strides only on the replica and group axes)
    for t, nm, inner in ((c, "clock", (1,)), (e, "ec", (A, 1)), (vc, "vclk", (V * A, A, 1)),
                         (vv, "vval", (V, 1))):
        if t.numel() and tuple(t.stride()[2:]) != inner:  # (an empty key shard: nothing is read)
            raise ValueError(f"map.lub_many: {nm} must be packed within a replica")
    Kw = (K + 63) // 64 if _key_shard is None else (int(_key_shard[1]) + 63) // 64
    dev = clock.device
    out_clock = torch.empty((G, A), dtype=torch.int64, device=dev)
    out_ec = torch.empty((G, K, A), dtype=torch.int64, device=dev)
    out_vc = torch.empty((G, K, vout, A), dtype=torch.int64, device=dev)
    out_vv = torch.empty((G, K, vout), dtype=torch.int64, device=dev)
    nval = torch.empty((G, K), dtype=torch.int32, device=dev)
    flags = torch.empty(G, dtype=torch.int32, device=dev)
    b = _abi.MapBatch()
    b.G, b.R, b.K, b.A, b.V = G, R, K, A, V
    b.clock, b.clock_rstride, b.clock_gstride = c.data_ptr(), c.stride(1), c.stride(0)
    b.ec, b.ec_rstride, b.ec_gstride = e.data_ptr(), e.stride(1), e.stride(0)
    b.vclk, b.vclk_rstride, b.vclk_gstride = vc.data_ptr(), vc.stride(1), vc.stride(0)
    b.vval, b.vval_rstride, b.vval_gstride = vv.data_ptr(), vv.stride(1), vv.stride(0)
    o = _abi.MapOut()
    o.Vout, o.Vstate = vout, vstate
    o.clock, o.ec, o.vclk, o.vval = out_clock.data_ptr(), out_ec.data_ptr(), out_vc.data_ptr(), out_vv.data_ptr()
    o.nval, o.flags = nval.data_ptr(), flags.data_ptr()
    keep = keys_out = None
    off_arr = None
    dev_off = isinstance(def_off, torch.Tensor) and def_off.device.type == "cuda"
    if dev_off:
        if (def_off.dtype not in (torch.int64, torch.uint64) or tuple(def_off.shape) != (G + 1,)
                or not def_off.is_contiguous() or def_off.device.index != ctx.device):
            raise ValueError(f"map.lub_many: a device def_off must be a contiguous ({G + 1},) int64 "
                             f"cuda:{ctx.device} tensor")
    if def_off is not None:
        if dev_off:
            D = 0 if def_clock is None else int(def_clock.shape[0])
        else:
            off = np.asarray(def_off, dtype=np.uint64)
            if off.shape != (G + 1,):
                raise ValueError(f"map.lub_many: def_off must have G+1 = {G + 1} entries")
            D = int(off[-1])
        if D > 0:
            for t, nm in ((def_clock, "def_clock"), (def_keys, "def_keys")):
                if t is None:
                    raise ValueError(f"map.lub_many: {nm} required with deferred removes")
                ctx.check_tensor(t, f"map.lub_many({nm})")
                if not t.is_contiguous():
                    raise ValueError(f"map.lub_many: {nm} must be contiguous")
            if def_row is None or def_row.dtype not in (torch.int32, torch.uint32) or not def_row.is_contiguous():
                raise ValueError("map.lub_many: def_row must be a contiguous int32 device tensor")
            if tuple(def_clock.shape) != (D, A) or tuple(def_keys.shape) != (D, Kw) or tuple(def_row.shape) != (D,):
                raise ValueError(f"map.lub_many: def_row {tuple(def_row.shape)} / def_clock "
                                 f"{tuple(def_clock.shape)} / def_keys {tuple(def_keys.shape)}; expected "
                                 f"({D},) / ({D},{A}) / ({D},{Kw})")
            if not dev_off:
                off_arr = (ctypes.c_size_t * (G + 1))(*[int(x) for x in off])
                b.def_off = ctypes.cast(off_arr, ctypes.POINTER(ctypes.c_size_t))
            b.def_row, b.def_clock, b.def_keys = def_row.data_ptr(), def_clock.data_ptr(), def_keys.data_ptr()
            keep = torch.empty(D, dtype=torch.uint8, device=dev)
            keys_out = torch.empty((D, Kw), dtype=torch.int64, device=dev)
            o.def_keep, o.def_keys = keep.data_ptr(), keys_out.data_ptr()
    if dev_off and _key_shard is None:
        ctx.call("crdt_map_lub_many_doff", ctypes.byref(b), def_off.data_ptr(), D, ctypes.byref(o))
    elif dev_off:  # key shard with device offsets (crdt_map_lub_many_sharded_doff)
        ctx.call("crdt_map_lub_many_sharded_doff", ctypes.byref(b), def_off.data_ptr(), D, int(_key_shard[0]),
                 int(_key_shard[1]), ctypes.byref(o))
    elif _key_shard is None:
        ctx.call("crdt_map_lub_many", ctypes.byref(b), ctypes.byref(o))
    else:
        ctx.call("crdt_map_lub_many_sharded", ctypes.byref(b), int(_key_shard[0]), int(_key_shard[1]),
                 ctypes.byref(o))
    if check:
        f = 0
        for x in flags.cpu().numpy().tolist():
            f |= int(x)
        if f & 2:
            raise ValueError("map.lub_many: def_row must be non-decreasing within each group and < R"
                             + (" (or the device def_off is invalid)" if dev_off else ""))
        if f & 8:
            raise RuntimeError("map.lub_many: internal fault (shared clock-row ring wait timed out)")
        # the fold state overflowed: rerun with the next larger state (a key-sharded call already
        # did that inside the C entry point, on every rank together)
        if f & 4 and vstate < 16 and _key_shard is None:
            return lub_many(clock, ec, vclk, vval, def_off, def_row, def_clock, def_keys, vout, ctx,
                            check, vstate=8 if vstate < 8 else 16, _key_shard=_key_shard)
        if f & 4 and (vstate >= 16 or _key_shard is not None):
            raise MapCapacityError("map.lub_many: a key held more than 16 MVReg values during the "
                                   "fold (the kernel's state capacity); results incomplete")
        if f & 1:
            raise MapCapacityError(f"map.lub_many: a key folds to more than vout={vout} values; "
                                   "retry with a larger vout")
    res = MapLub(out_clock, out_ec, out_vc, out_vv, nval, flags, keep, keys_out)
    if squeeze:
        res = MapLub(out_clock[0], out_ec[0], out_vc[0], out_vv[0], nval[0], flags, keep, keys_out)
    return res


def deferred_set(def_clock: torch.Tensor, def_keep: torch.Tensor, def_keys: torch.Tensor,
                 lo: int = 0, hi: Optional[int] = None) -> set:
    """Egress of the surviving deferred removes: {(rm clock tuple, frozenset of key indices)}."""
    from .orswot import deferred_set as _ds
    return _ds(def_clock, def_keep, def_keys, lo, hi)


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


def forget_batch(clock: torch.Tensor, ec: torch.Tensor, vclk: torch.Tensor, vval: torch.Tensor, y: torch.Tensor,
                 def_clock: Optional[torch.Tensor] = None, def_state: Optional[torch.Tensor] = None,
                 ctx: Optional[Context] = None) -> Optional[torch.Tensor]:
    """Causal::forget of N Map<K, MVReg> states in place (map.rs:85-114, mvreg.rs:88-104):
    clock (N, A), ec (N, K, A), vclk (N, K, V, A), vval (N, K, V), y (A,) or (N, A); deferred as
    for orswot.forget_batch.  Returns def_keep or None."""
    ctx = ctx or Context.default(clock.device.index)
    for t, nm in ((clock, "clock"), (ec, "ec"), (vclk, "vclk"), (vval, "vval")):
        ctx.check_tensor(t, f"map.forget_batch({nm})")
    if clock.dim() != 2 or ec.dim() != 3 or vclk.dim() != 4 or vval.dim() != 3:
        raise ValueError("map.forget_batch: clock (N,A), ec (N,K,A), vclk (N,K,V,A), vval (N,K,V) expected")
    N, A = clock.shape
    K, V = vclk.shape[1], vclk.shape[2]
    if (tuple(ec.shape) != (N, K, A) or tuple(vclk.shape) != (N, K, V, A) or tuple(vval.shape) != (N, K, V)
            or clock.stride(1) != 1 or ec.stride(2) != 1 or ec.stride(1) != A or vclk.stride(3) != 1
            or vclk.stride(2) != A or vclk.stride(1) != V * A or vval.stride(2) != 1 or vval.stride(1) != V):
        raise ValueError("map.forget_batch: per-state blocks must be packed (K, A) / (K, V, A) / (K, V)")
    y, ys = _forget_clock(ctx, y, N, A, "map.forget_batch(y)")
    dp, sp, D, keep = _forget_deferred(ctx, def_clock, def_state, N, A, "map.forget_batch(def_clock)")
    st = _abi.MapStates()
    st.N, st.K, st.A, st.V = N, K, A, V
    st.clock, st.clock_stride = clock.data_ptr(), clock.stride(0)
    st.ec, st.ec_stride = ec.data_ptr(), ec.stride(0)
    st.vclk, st.vclk_stride = vclk.data_ptr(), vclk.stride(0)
    st.vval, st.vval_stride = vval.data_ptr(), vval.stride(0)
    ctx.call("crdt_map_forget_batch", ctypes.byref(st), y.data_ptr(), ys, dp, sp, D,
             keep.data_ptr() if keep is not None else None)
    return keep


# ---------------------------------------------------------------------------------------------
# Batched CmRDT::apply (map.rs:119-137, apply_keyset_rm :318-348, MVReg::apply mvreg.rs:130-166)
# ---------------------------------------------------------------------------------------------
class MapOpBatch(NamedTuple):
    """Device op streams (crdt_map_ops): state s applies ops [op_off[s], op_off[s+1]) in order."""
    op_off: torch.Tensor    # (N+1,) int64
    kind: torch.Tensor      # (n_ops,) uint8: 0 = Op::Up, 1 = Op::Rm
    actor: torch.Tensor     # (n_ops,) int32   Up: dot.actor
    counter: torch.Tensor   # (n_ops,) int64   Up: dot.counter
    key: torch.Tensor       # (n_ops,) int32   Up: key
    val: torch.Tensor       # (n_ops,) int64   Up: Put.val
    clk_row: torch.Tensor   # (n_ops,) int32   row of clk_pool: Put.clock (Up) / rm clock (Rm)
    clk_pool: torch.Tensor  # (n_clk, A) int64
    key_off: torch.Tensor   # (n_ops+1,) int64 Rm keysets
    keys: torch.Tensor      # (n_keys,) int32


def encode_ops(streams, A: int, device) -> MapOpBatch:
    """Host ingest of per-state op streams (interned to dense indices): ("up", actor, counter,
    key, put_clock, val) for Op::Up { dot, key, op: MVReg Op::Put { clock, val } } or
    ("rm", clock, keys) for Op::Rm { clock, keyset } (map.rs:51-66, mvreg.rs:38-47); clocks are
    mappings actor -> counter or dense rows of A counters."""
    def row(clk):
        r = np.zeros(A, dtype=np.uint64)
        if hasattr(clk, "items"):
            for a, c in clk.items():
                r[int(a)] = np.uint64(c)
        else:
            r[:] = np.asarray(clk, dtype=np.uint64)
        return r

    op_off, kind, actor, counter, key, val, clk_row, key_off, keys, pool = [0], [], [], [], [], [], [], [0], [], []
    for ops in streams:
        for op in ops:
            if op[0] == "up":
                _, a, k, kk, pc, v = op
                kind.append(0)
                actor.append(int(a))
                counter.append(int(k))
                key.append(int(kk))
                val.append(int(v))
                clk_row.append(len(pool))
                pool.append(row(pc))
            elif op[0] == "rm":
                _, rc, ks = op
                kind.append(1)
                actor.append(0)
                counter.append(0)
                key.append(0)
                val.append(0)
                clk_row.append(len(pool))
                pool.append(row(rc))
                keys.extend(int(x) for x in ks)
            else:
                raise ValueError(f"map.encode_ops: unknown op {op[0]!r}")
            key_off.append(len(keys))
        op_off.append(len(kind))
    pool.append(np.zeros(A, dtype=np.uint64))  # pads: never-empty device buffers
    keys.append(0)

    def t(x, dt):
        return torch.from_numpy(np.asarray(x, dtype=dt)).to(device)

    u64 = lambda x: t(np.array(x, dtype=np.uint64).view(np.int64), np.int64)  # noqa: E731
    return MapOpBatch(t(op_off, np.int64), t(kind, np.uint8), t(actor, np.int32), u64(counter), t(key, np.int32),
                      u64(val), t(clk_row, np.int32),
                      torch.from_numpy(np.stack(pool).view(np.int64)).to(device), t(key_off, np.int64),
                      t(keys, np.int32))


def apply_batch(clock: torch.Tensor, ec: torch.Tensor, vclk: torch.Tensor, vval: torch.Tensor,
                def_clock: torch.Tensor, def_keys: torch.Tensor, def_count: torch.Tensor, ops: MapOpBatch,
                ctx: Optional[Context] = None) -> torch.Tensor:
    """Apply every state's op stream in place: clock (N, A), ec (N, K, A), vclk (N, K, V, A),
    vval (N, K, V), deferred slots def_clock (N, Dcap, A) / def_keys (N, Dcap, ceil(K/64)) /
    def_count (N,) int32.  Returns the per-state status (N,) int32 (include/crdt_gpu.h)."""
    ctx = ctx or Context.default(clock.device.index)
    for t_, nm in ((clock, "clock"), (ec, "ec"), (vclk, "vclk"), (vval, "vval"), (def_clock, "def_clock"),
                   (def_keys, "def_keys")):
        ctx.check_tensor(t_, f"map.apply_batch({nm})")
    N, A = clock.shape
    K, V = vclk.shape[1], vclk.shape[2]
    Kw = (K + 63) // 64
    Dcap = def_clock.shape[1]
    if (tuple(ec.shape) != (N, K, A) or tuple(vclk.shape) != (N, K, V, A) or tuple(vval.shape) != (N, K, V)
            or clock.stride(1) != 1 or ec.stride(2) != 1 or ec.stride(1) != A or vclk.stride(3) != 1
            or vclk.stride(2) != A or vclk.stride(1) != V * A or vval.stride(2) != 1 or vval.stride(1) != V):
        raise ValueError("map.apply_batch: per-state blocks must be packed (K, A) / (K, V, A) / (K, V)")
    if (tuple(def_clock.shape) != (N, Dcap, A) or tuple(def_keys.shape) != (N, Dcap, Kw)
            or not def_clock.is_contiguous() or not def_keys.is_contiguous()):
        raise ValueError("map.apply_batch: def_clock / def_keys must be contiguous (N, Dcap, A) / (N, Dcap, Kw)")
    want = {"op_off": (torch.int64,), "kind": (torch.uint8,), "actor": (torch.int32,), "counter": (torch.int64,),
            "key": (torch.int32,), "val": (torch.int64,), "clk_row": (torch.int32,), "clk_pool": (torch.int64,),
            "key_off": (torch.int64,), "keys": (torch.int32,)}
    for nm, t_ in list(zip(ops._fields, ops)) + [("def_count", def_count)]:
        dts = want.get(nm, (torch.int32,))
        if t_.device.type != "cuda" or t_.device.index != ctx.device or t_.dtype not in dts or not t_.is_contiguous():
            raise ValueError(f"map.apply_batch({nm}): expected a contiguous cuda:{ctx.device} tensor of {dts}")
    n = ops.kind.shape[0]
    if (ops.op_off.shape[0] != N + 1 or ops.key_off.shape[0] != n + 1 or ops.clk_pool.dim() != 2
            or ops.clk_pool.shape[1] != A or tuple(def_count.shape) != (N,)):
        raise ValueError("map.apply_batch: op_off (N+1,), key_off (n_ops+1,), clk_pool (n, A), def_count (N,)")
    for nm in ("actor", "counter", "key", "val", "clk_row"):
        if getattr(ops, nm).shape[0] != n:
            raise ValueError(f"map.apply_batch: ops.{nm} must have n_ops entries")
    st = _abi.MapStates()
    st.N, st.K, st.A, st.V = N, K, A, V
    st.clock, st.clock_stride = clock.data_ptr(), clock.stride(0)
    st.ec, st.ec_stride = ec.data_ptr(), ec.stride(0)
    st.vclk, st.vclk_stride = vclk.data_ptr(), vclk.stride(0)
    st.vval, st.vval_stride = vval.data_ptr(), vval.stride(0)
    o = _abi.MapOps()
    o.n_ops = n
    o.op_off, o.kind, o.actor, o.counter = (ops.op_off.data_ptr(), ops.kind.data_ptr(), ops.actor.data_ptr(),
                                            ops.counter.data_ptr())
    o.key, o.val, o.clk_row, o.clk_pool = ops.key.data_ptr(), ops.val.data_ptr(), ops.clk_row.data_ptr(), \
        ops.clk_pool.data_ptr()
    o.n_clk_rows, o.key_off, o.keys = ops.clk_pool.shape[0], ops.key_off.data_ptr(), ops.keys.data_ptr()
    o.n_keys = ops.keys.shape[0]
    status = torch.empty(N, dtype=torch.int32, device=clock.device)
    ctx.call("crdt_map_apply_batch", ctypes.byref(st), def_clock.data_ptr(), def_keys.data_ptr(),
             def_count.data_ptr(), Dcap, ctypes.byref(o), status.data_ptr())
    return status


# ---------------------------------------------------------------------------------------------
# Pairwise in-place merge_batch: self[i].merge(other[i]) (map.rs:140-220)
# ---------------------------------------------------------------------------------------------
class MapStates(NamedTuple):
    """N Map<K, MVReg<u64>> states: the apply_batch layout plus deferred slots."""
    clock: torch.Tensor      # (N, A)
    ec: torch.Tensor         # (N, K, A)
    vclk: torch.Tensor       # (N, K, V, A)
    vval: torch.Tensor       # (N, K, V)
    def_clock: torch.Tensor  # (N, Dcap, A)
    def_keys: torch.Tensor   # (N, Dcap, ceil(K/64))
    def_count: torch.Tensor  # (N,) int32


def _map_states_structs(ctx: Context, st: MapStates, what: str):
    for t, nm in zip(st, st._fields):
        if nm != "def_count":
            ctx.check_tensor(t, f"{what}({nm})")
    N, A = st.clock.shape
    K, V = st.ec.shape[1], st.vclk.shape[2]
    Kw = (K + 63) // 64
    Dcap = st.def_clock.shape[1]
    if (tuple(st.ec.shape) != (N, K, A) or tuple(st.vclk.shape) != (N, K, V, A) or tuple(st.vval.shape) != (N, K, V)
            or st.clock.stride(1) != 1 or st.ec.stride(2) != 1 or st.ec.stride(1) != A or st.vclk.stride(3) != 1
            or st.vclk.stride(2) != A or st.vclk.stride(1) != V * A or st.vval.stride(2) != 1 or st.vval.stride(1) != V):
        raise ValueError(f"{what}: per-state blocks must be packed (K, A) / (K, V, A) / (K, V)")
    if (tuple(st.def_clock.shape) != (N, Dcap, A) or tuple(st.def_keys.shape) != (N, Dcap, Kw)
            or not st.def_clock.is_contiguous() or not st.def_keys.is_contiguous()):
        raise ValueError(f"{what}: def_clock / def_keys must be contiguous (N, Dcap, A) / (N, Dcap, Kw)")
    if (st.def_count.dtype not in (torch.int32, torch.uint32) or tuple(st.def_count.shape) != (N,)
            or st.def_count.device != st.clock.device):
        raise ValueError(f"{what}: def_count must be an (N,) int32 tensor on the states' device")
    s = _abi.MapStates()
    s.N, s.K, s.A, s.V = N, K, A, V
    s.clock, s.clock_stride = st.clock.data_ptr(), st.clock.stride(0)
    s.ec, s.ec_stride = st.ec.data_ptr(), st.ec.stride(0)
    s.vclk, s.vclk_stride = st.vclk.data_ptr(), st.vclk.stride(0)
    s.vval, s.vval_stride = st.vval.data_ptr(), st.vval.stride(0)
    d = _abi.MapDeferred()
    d.clock, d.keys, d.count, d.Dcap = st.def_clock.data_ptr(), st.def_keys.data_ptr(), st.def_count.data_ptr(), Dcap
    return s, d


def merge_batch(self_states: MapStates, other: MapStates, ctx: Optional[Context] = None) -> torch.Tensor:
    """self[i].merge(other[i]) for every i, in place on `self_states` (Map::merge map.rs:140-220 with
    MVReg::merge mvreg.rs:112-128), exact for any pair of states.  Returns status (N,) int32:
    bit 0 = deferred slots exhausted, bit 2 = invalid def_count, bit 4 = a register needed more
    than self's V value slots."""
    ctx = ctx or Context.default(self_states.clock.device.index)
    a, ad = _map_states_structs(ctx, self_states, "map.merge_batch(self)")
    b, bd = _map_states_structs(ctx, other, "map.merge_batch(other)")
    if (a.N, a.K, a.A) != (b.N, b.K, b.A):
        raise ValueError("map.merge_batch: self and other differ in N, K or A")
    status = torch.empty(a.N, dtype=torch.int32, device=self_states.clock.device)
    ctx.call("crdt_map_merge_batch", ctypes.byref(a), ctypes.byref(ad), ctypes.byref(b), ctypes.byref(bd),
             status.data_ptr())
    return status


# ---- Map<K, GCounter> / Map<K, PNCounter> (crdt_map_counter_lub_many, round 4) ----------------------
class MapCounterLub(NamedTuple):
    clock: torch.Tensor               # (G, A)
    ec: torch.Tensor                  # (G, K, A)
    val: torch.Tensor                 # (G, K, W, A): GCounter row (W = 1) or P, N rows (W = 2)
    flags: torch.Tensor               # (G,) int32
    def_keep: Optional[torch.Tensor]  # (D,) uint8
    def_keys: Optional[torch.Tensor]  # (D, Kw)


def counter_lub_many(clock: torch.Tensor, ec: torch.Tensor, val: torch.Tensor, def_off=None,
                     def_row: Optional[torch.Tensor] = None, def_clock: Optional[torch.Tensor] = None,
                     def_keys: Optional[torch.Tensor] = None, ctx: Optional[Context] = None,
                     check: bool = True, _key_shard: Optional[tuple] = None) -> MapCounterLub:
    """The exact left fold of Map::merge (map.rs:140-220) for Map<K, GCounter> (val (G,R,K,1,A)) or
    Map<K, PNCounter> (val (G,R,K,2,A): P then N) — gcounter.rs:44-54 / pncounter.rs:70-82 as the
    value's merge and forget.  clock (G,R,A) / (R,A), ec (G,R,K,A) / (R,K,A), val likewise; the
    deferred pool as for lub_many (host def_off).  check=True raises on flags (bit 1: def_row not
    sorted / out of range, bit 3: more than 512 live removes named one key)."""
    ctx = ctx or Context.default(clock.device.index)
    for t, nm in ((clock, "clock"), (ec, "ec"), (val, "val")):
        ctx.check_tensor(t, f"map.counter_lub_many({nm})")
    squeeze = clock.dim() == 2
    c = clock.unsqueeze(0) if squeeze else clock
    e = ec.unsqueeze(0) if squeeze else ec
    v = val.unsqueeze(0) if squeeze else val
    if c.dim() != 3 or e.dim() != 4 or v.dim() != 5:
        raise ValueError("map.counter_lub_many: clock (G,R,A), ec (G,R,K,A), val (G,R,K,W,A) expected")
    G, R, A = c.shape
    K, W = e.shape[2], v.shape[3]
    if tuple(e.shape) != (G, R, K, A) or tuple(v.shape) != (G, R, K, W, A) or W not in (1, 2):
        raise ValueError(f"map.counter_lub_many: shapes clock {tuple(c.shape)} ec {tuple(e.shape)} "
                         f"val {tuple(v.shape)} do not agree (W = 1 GCounter, 2 PNCounter)")
    for t, nm, inner in ((c, "clock", (1,)), (e, "ec", (A, 1)), (v, "val", (W * A, A, 1))):
        if t.numel() and tuple(t.stride()[2:]) != inner:
            raise ValueError(f"map.counter_lub_many: {nm} must be packed within a replica")
    Kw = (K + 63) // 64 if _key_shard is None else (int(_key_shard[1]) + 63) // 64
    dev = clock.device
    out_clock = torch.empty((G, A), dtype=torch.int64, device=dev)
    out_ec = torch.empty((G, K, A), dtype=torch.int64, device=dev)
    out_val = torch.empty((G, K, W, A), dtype=torch.int64, device=dev)
    flags = torch.empty(G, dtype=torch.int32, device=dev)
    b = _abi.MapCounterBatch()
    b.G, b.R, b.K, b.A, b.W = G, R, K, A, W
    b.clock, b.clock_rstride, b.clock_gstride = c.data_ptr(), c.stride(1), c.stride(0)
    b.ec, b.ec_rstride, b.ec_gstride = e.data_ptr(), e.stride(1), e.stride(0)
    b.val, b.val_rstride, b.val_gstride = v.data_ptr(), v.stride(1), v.stride(0)
    o = _abi.MapCounterOut()
    o.clock, o.ec, o.val, o.flags = out_clock.data_ptr(), out_ec.data_ptr(), out_val.data_ptr(), flags.data_ptr()
    keep = keys_out = None
    off_arr = None
    if def_off is not None:
        off = np.asarray(def_off, dtype=np.uint64)
        if off.shape != (G + 1,):
            raise ValueError(f"map.counter_lub_many: def_off must have G+1 = {G + 1} entries")
        D = int(off[-1])
        if D > 0:
            for t, nm, shape in ((def_clock, "def_clock", (D, A)), (def_keys, "def_keys", (D, Kw)),
                                 (def_row, "def_row", (D,))):
                if t is None or not t.is_contiguous() or tuple(t.shape) != shape:
                    raise ValueError(f"map.counter_lub_many: {nm} must be a contiguous {shape} tensor")
                if nm != "def_row":
                    ctx.check_tensor(t, f"map.counter_lub_many({nm})")
            if def_row.dtype not in (torch.int32, torch.uint32) or def_row.device != dev:
                raise ValueError(f"map.counter_lub_many: def_row must be an int32 tensor on {dev}")
            off_arr = (ctypes.c_size_t * (G + 1))(*[int(x) for x in off])
            b.def_off = ctypes.cast(off_arr, ctypes.POINTER(ctypes.c_size_t))
            b.def_row, b.def_clock, b.def_keys = def_row.data_ptr(), def_clock.data_ptr(), def_keys.data_ptr()
            keep = torch.empty(D, dtype=torch.uint8, device=dev)
            keys_out = torch.empty((D, Kw), dtype=torch.int64, device=dev)
            o.def_keep, o.def_keys = keep.data_ptr(), keys_out.data_ptr()
    if _key_shard is None:
        ctx.call("crdt_map_counter_lub_many", ctypes.byref(b), ctypes.byref(o))
    else:  # (shard.map_counter_lub_many_sharded: this rank's keys of a key-sharded fold)
        ctx.call("crdt_map_counter_lub_many_sharded", ctypes.byref(b), int(_key_shard[0]), int(_key_shard[1]),
                 ctypes.byref(o))
    if check:
        f = 0
        for x in flags.cpu().numpy().tolist():
            f |= int(x)
        if f & 2:
            raise ValueError("map.counter_lub_many: def_row not non-decreasing per group or >= R")
        if f & 8:
            raise RuntimeError("map.counter_lub_many: more than 512 live removes named one key")
    if squeeze:
        out_clock, out_ec, out_val, flags = out_clock[0], out_ec[0], out_val[0], flags
    return MapCounterLub(out_clock, out_ec, out_val, flags, keep, keys_out)


# ---- Map<K, Orswot<M>> (crdt_map_orswot_lub_many, round 4) ------------------------------------------
VD_CAP = 16  # nested deferred removes per key state by default (crdt_gpu.h; round 6: any Vd >= 16)


class MapOrswotLub(NamedTuple):
    clock: torch.Tensor               # (G, A)
    ec: torch.Tensor                  # (G, K, A)
    oc: torch.Tensor                  # (G, K, A) the nested Orswot clocks
    ent: torch.Tensor                 # (G, K, M, A) its member dots
    vd_n: torch.Tensor                # (G, K) int32: nested deferred removes per key
    vd_clock: torch.Tensor            # (G, K, Vd, A)  (Vd = vd_cap, 16 by default)
    vd_mem: torch.Tensor              # (G, K, Vd) member bitmasks ((G, K, Vd, Mw) past M = 64)
    flags: torch.Tensor               # (G,) int32
    def_keep: Optional[torch.Tensor]  # (D,) uint8
    def_keys: Optional[torch.Tensor]  # (D, Kw)


def orswot_lub_many(clock: torch.Tensor, ec: torch.Tensor, oc: torch.Tensor, ent: torch.Tensor,
                    vd_off: torch.Tensor, vd_clock: Optional[torch.Tensor] = None,
                    vd_mem: Optional[torch.Tensor] = None, def_off=None, def_row: Optional[torch.Tensor] = None,
                    def_clock: Optional[torch.Tensor] = None, def_keys: Optional[torch.Tensor] = None,
                    ctx: Optional[Context] = None, check: bool = True,
                    _key_shard: Optional[tuple] = None, vd_cap=VD_CAP) -> MapOrswotLub:
    """The exact left fold of Map::merge (map.rs:140-220) for Map<K, Orswot<M>> — orswot.rs:81-149 as
    the value's merge, :150-183 as its forget.  clock (G,R,A) / (R,A), ec and oc (G,R,K,A), ent
    (G,R,K,M,A), all contiguous; the nested deferred removes as a device CSR over (g, r, k): vd_off
    (G*R*K + 1,) int64, vd_clock (Dv, A), vd_mem (Dv,) member bitmasks ((Dv, Mw) words, Mw = ceil(M/64),
    past M = 64); the Map's own deferred pool as for lub_many (host def_off).  A <= 1,024, M <= 1,024
    (past A = 64 or M = 32 the library runs its wide kernel).  check=True raises on flags (bit 1: def_row not sorted / out of
    range, bit 3: more than 256 live Map removes named one key, bit 4: more than vd_cap nested deferred
    removes on one key).  vd_cap: nested slots per key in the result (>= 16; round 6: the fold keeps 16
    in LDS and re-folds exactly the keys that need more); "auto" sizes it to the largest sum of one
    key's nested list lengths over its group's replicas, a bound no fold result can pass."""
    ctx = ctx or Context.default(clock.device.index)
    squeeze = clock.dim() == 2
    c, e, o, m = ((t.unsqueeze(0) if squeeze else t) for t in (clock, ec, oc, ent))
    if c.dim() != 3 or e.dim() != 4 or o.dim() != 4 or m.dim() != 5:
        raise ValueError("map.orswot_lub_many: clock (G,R,A), ec / oc (G,R,K,A), ent (G,R,K,M,A) expected")
    G, R, A = c.shape
    K, M = e.shape[2], m.shape[3]
    if tuple(e.shape) != (G, R, K, A) or tuple(o.shape) != (G, R, K, A) or tuple(m.shape) != (G, R, K, M, A):
        raise ValueError(f"map.orswot_lub_many: shapes clock {tuple(c.shape)} ec {tuple(e.shape)} oc "
                         f"{tuple(o.shape)} ent {tuple(m.shape)} do not agree")
    for t, nm in ((c, "clock"), (e, "ec"), (o, "oc"), (m, "ent")):
        ctx.check_tensor(t, f"map.orswot_lub_many({nm})")
        if not t.is_contiguous():
            raise ValueError(f"map.orswot_lub_many: {nm} must be contiguous")
    dev = clock.device
    if vd_off.device != dev or not vd_off.is_contiguous() or tuple(vd_off.shape) != (G * R * K + 1,):
        raise ValueError(f"map.orswot_lub_many: vd_off must be a contiguous ({G * R * K + 1},) tensor on {dev}")
    if vd_off.dtype not in (torch.int64, torch.uint64):
        raise ValueError(f"map.orswot_lub_many: vd_off must be int64 / uint64 (got {vd_off.dtype})")
    # Dv = rows of vd_clock / vd_mem; the library checks vd_off against it on the device (flags bit 5)
    Dv = int(vd_clock.shape[0]) if vd_clock is not None else 0
    Mw = max(1, (M + 63) // 64)
    if Dv > 0:
        for t, nm, shape in ((vd_clock, "vd_clock", (Dv, A)), (vd_mem, "vd_mem", (Dv,) if Mw == 1 else (Dv, Mw))):
            if t is None or not t.is_contiguous() or tuple(t.shape) not in (shape, (Dv, 1) if Mw == 1 else shape):
                raise ValueError(f"map.orswot_lub_many: {nm} must be a contiguous {shape} tensor")
            ctx.check_tensor(t, f"map.orswot_lub_many({nm})")
    Kw = (K + 63) // 64 if _key_shard is None else (int(_key_shard[1]) + 63) // 64
    if vd_cap == "auto":
        lens = vd_off.view(torch.int64).reshape(-1)
        lens = (lens[1:] - lens[:-1]).clamp(min=0).reshape(G, R, K).sum(dim=1)
        vd_cap = max(VD_CAP, int(lens.max().item()) if lens.numel() else 0)
    Vd = int(vd_cap)
    if Vd < VD_CAP:
        raise ValueError(f"map.orswot_lub_many: vd_cap = {Vd} < {VD_CAP}")
    out = [torch.empty(sh, dtype=torch.int64, device=dev)
           for sh in ((G, A), (G, K, A), (G, K, A), (G, K, M, A), (G, K, Vd, A),
                      (G, K, Vd) if Mw == 1 else (G, K, Vd, Mw))]
    vd_n = torch.empty((G, K), dtype=torch.int32, device=dev)
    flags = torch.empty(G, dtype=torch.int32, device=dev)
    b = _abi.MapOrswotBatch()
    b.G, b.R, b.K, b.M, b.A = G, R, K, M, A
    b.clock, b.ec, b.oc, b.ent = c.data_ptr(), e.data_ptr(), o.data_ptr(), m.data_ptr()
    b.vd_off, b.Dv = vd_off.data_ptr(), Dv
    if Dv > 0:
        b.vd_clock, b.vd_mem = vd_clock.data_ptr(), vd_mem.data_ptr()
    ob = _abi.MapOrswotOut()
    ob.clock, ob.ec, ob.oc, ob.ent, ob.vd_clock, ob.vd_mem = (t.data_ptr() for t in out)
    ob.vd_n, ob.flags, ob.Vd = vd_n.data_ptr(), flags.data_ptr(), Vd
    keep = keys_out = None
    off_arr = None
    if def_off is not None:
        off = np.asarray(def_off, dtype=np.uint64)
        if off.shape != (G + 1,):
            raise ValueError(f"map.orswot_lub_many: def_off must have G+1 = {G + 1} entries")
        D = int(off[-1])
        if D > 0:
            for t, nm, shape in ((def_clock, "def_clock", (D, A)), (def_keys, "def_keys", (D, Kw)),
                                 (def_row, "def_row", (D,))):
                if t is None or not t.is_contiguous() or tuple(t.shape) != shape:
                    raise ValueError(f"map.orswot_lub_many: {nm} must be a contiguous {shape} tensor")
                if nm != "def_row":
                    ctx.check_tensor(t, f"map.orswot_lub_many({nm})")
            if def_row.dtype not in (torch.int32, torch.uint32) or def_row.device != dev:
                raise ValueError(f"map.orswot_lub_many: def_row must be an int32 tensor on {dev}")
            off_arr = (ctypes.c_size_t * (G + 1))(*[int(x) for x in off])
            b.def_off = ctypes.cast(off_arr, ctypes.POINTER(ctypes.c_size_t))
            b.def_row, b.def_clock, b.def_keys = def_row.data_ptr(), def_clock.data_ptr(), def_keys.data_ptr()
            keep = torch.empty(D, dtype=torch.uint8, device=dev)
            keys_out = torch.empty((D, Kw), dtype=torch.int64, device=dev)
            ob.def_keep, ob.def_keys = keep.data_ptr(), keys_out.data_ptr()
    if _key_shard is None:
        ctx.call("crdt_map_orswot_lub_many", ctypes.byref(b), ctypes.byref(ob))
    else:  # (shard.map_orswot_lub_many_sharded)
        ctx.call("crdt_map_orswot_lub_many_sharded", ctypes.byref(b), int(_key_shard[0]), int(_key_shard[1]),
                 ctypes.byref(ob))
    if check:
        f = 0
        for x in flags.cpu().numpy().tolist():
            f |= int(x)
        if f & 2:
            raise ValueError("map.orswot_lub_many: def_row not non-decreasing per group or >= R")
        if f & 8:
            raise RuntimeError("map.orswot_lub_many: more live removes named one key than the deep pass holds")
        if f & 32:
            raise ValueError("map.orswot_lub_many: vd_off invalid (must start at 0, be non-decreasing and end at "
                             "vd_clock.shape[0])")
        if f & 16:
            raise RuntimeError(f"map.orswot_lub_many: more than vd_cap = {Vd} deferred removes in one key's Orswot "
                               "(vd_cap='auto' always fits)")
    oclk, oec, ooc, oent, ovdc, ovdm = out
    if squeeze:
        oclk, oec, ooc, oent, vd_n, ovdc, ovdm = oclk[0], oec[0], ooc[0], oent[0], vd_n[0], ovdc[0], ovdm[0]
    return MapOrswotLub(oclk, oec, ooc, oent, vd_n, ovdc, ovdm, flags, keep, keys_out)


# ---- Map<K, Map<K2, MVReg<u64>>> (crdt_map_nested_lub_many, round 5) -------------------------------
NM_VS = 8   # MVReg slots per inner key in the fold state by default (round 6: any Vs in 8..64)
NM_ID = 16  # inner deferred removes per key state by default (round 6: any Id >= 16)


class MapNestedLub(NamedTuple):
    clock: torch.Tensor               # (G, A)
    ec: torch.Tensor                  # (G, K, A) outer entry clocks
    ic: torch.Tensor                  # (G, K, A) inner Map clocks
    iec: torch.Tensor                 # (G, K, K2, A) inner entry clocks
    ivc: torch.Tensor                 # (G, K, K2, Vs, A) inner MVReg slot clocks (Vs = v_cap, 8 by default)
    ivv: torch.Tensor                 # (G, K, K2, Vs) values
    nval: torch.Tensor                # (G, K, K2) int32 slots used
    id_n: torch.Tensor                # (G, K) int32 inner deferred removes
    id_clock: torch.Tensor            # (G, K, Id, A)  (Id = id_cap, 16 by default)
    id_keys: torch.Tensor             # (G, K, Id) inner key bitmasks ((G, K, Id, K2w) past K2 = 64)
    flags: torch.Tensor               # (G,) int32
    def_keep: Optional[torch.Tensor]  # (D,) uint8
    def_keys: Optional[torch.Tensor]  # (D, Kw)


def nested_lub_many(clock: torch.Tensor, ec: torch.Tensor, ic: torch.Tensor, iec: torch.Tensor, ivc: torch.Tensor,
                    ivv: torch.Tensor, id_off: torch.Tensor, id_clock: Optional[torch.Tensor] = None,
                    id_keys: Optional[torch.Tensor] = None, def_off=None, def_row: Optional[torch.Tensor] = None,
                    def_clock: Optional[torch.Tensor] = None, def_keys: Optional[torch.Tensor] = None,
                    ctx: Optional[Context] = None, check: bool = True,
                    _key_shard: Optional[tuple] = None, id_cap=NM_ID, v_cap: int = NM_VS) -> MapNestedLub:
    """The exact left fold of Map::merge (map.rs:140-220) for Map<K, Map<K2, MVReg<u64>>> — the type of
    the reference's own Map tests (test/map.rs:10) — with the inner Map's merge (map.rs:140-220,
    mvreg.rs:112-128) and forget (map.rs:85-114) as the value's.  clock (G,R,A) / (R,A); ec, ic
    (G,R,K,A); iec (G,R,K,K2,A); ivc (G,R,K,K2,V,A); ivv (G,R,K,K2,V), all contiguous; the inner
    deferred removes as a device CSR over (g, r, k): id_off (G*R*K + 1,) int64, id_clock (Di, A),
    id_keys (Di,) inner-key bitmasks ((Di, K2w) words past K2 = 64; K2 <= 256, A <= 256); the outer
    deferred pool as for lub_many (host def_off).
    check=True raises on flags (bit 1: def_row unsorted / out of range, bit 3: more than 256 live outer
    removes named one key, bit 4: more than id_cap inner deferred removes, bit 5: id_off invalid, bit 6:
    more than 8 values on one inner key).  id_cap: inner deferred slots per key in the result (>= 16;
    round 6: the fold keeps 16 in LDS and re-folds exactly the keys that need more); "auto" sizes it to
    the largest sum of one key's inner list lengths over its group's replicas.  v_cap: MVReg slots per
    inner key in the result (8..64; round 6: keys past 8 values re-fold in the deep pass, which also
    takes inputs with V up to 64)."""
    ctx = ctx or Context.default(clock.device.index)
    squeeze = clock.dim() == 2
    c, e, i, ie, vc, vv = ((t.unsqueeze(0) if squeeze else t) for t in (clock, ec, ic, iec, ivc, ivv))
    if c.dim() != 3 or e.dim() != 4 or i.dim() != 4 or ie.dim() != 5 or vc.dim() != 6 or vv.dim() != 5:
        raise ValueError("map.nested_lub_many: clock (G,R,A), ec / ic (G,R,K,A), iec (G,R,K,K2,A), "
                         "ivc (G,R,K,K2,V,A), ivv (G,R,K,K2,V) expected")
    G, R, A = c.shape
    K, K2, V = e.shape[2], ie.shape[3], vc.shape[4]
    if (tuple(e.shape) != (G, R, K, A) or tuple(i.shape) != (G, R, K, A) or tuple(ie.shape) != (G, R, K, K2, A)
            or tuple(vc.shape) != (G, R, K, K2, V, A) or tuple(vv.shape) != (G, R, K, K2, V)):
        raise ValueError("map.nested_lub_many: shapes do not agree")
    for t, nm in ((c, "clock"), (e, "ec"), (i, "ic"), (ie, "iec"), (vc, "ivc"), (vv, "ivv")):
        ctx.check_tensor(t, f"map.nested_lub_many({nm})")
        if not t.is_contiguous():
            raise ValueError(f"map.nested_lub_many: {nm} must be contiguous")
    dev = clock.device
    if id_off.device != dev or not id_off.is_contiguous() or tuple(id_off.shape) != (G * R * K + 1,):
        raise ValueError(f"map.nested_lub_many: id_off must be a contiguous ({G * R * K + 1},) tensor on {dev}")
    if id_off.dtype not in (torch.int64, torch.uint64):
        raise ValueError(f"map.nested_lub_many: id_off must be int64 / uint64 (got {id_off.dtype})")
    Di = int(id_clock.shape[0]) if id_clock is not None else 0
    K2w = max(1, (K2 + 63) // 64)
    if Di > 0:
        for t, nm, shapes in ((id_clock, "id_clock", ((Di, A),)),
                              (id_keys, "id_keys", ((Di,), (Di, 1)) if K2w == 1 else ((Di, K2w),))):
            if t is None or not t.is_contiguous() or tuple(t.shape) not in shapes:
                raise ValueError(f"map.nested_lub_many: {nm} must be a contiguous {shapes[0]} tensor")
            ctx.check_tensor(t, f"map.nested_lub_many({nm})")
    Kw = (K + 63) // 64 if _key_shard is None else (int(_key_shard[1]) + 63) // 64
    if id_cap == "auto":
        lens = id_off.view(torch.int64).reshape(-1)
        lens = (lens[1:] - lens[:-1]).clamp(min=0).reshape(G, R, K).sum(dim=1)
        id_cap = max(NM_ID, int(lens.max().item()) if lens.numel() else 0)
    Id = int(id_cap)
    Vs = int(v_cap)
    if not NM_VS <= Vs <= 64 or Vs < V:
        raise ValueError(f"map.nested_lub_many: v_cap = {Vs} outside {max(NM_VS, V)}..64")
    if Id < NM_ID:
        raise ValueError(f"map.nested_lub_many: id_cap = {Id} < {NM_ID}")
    out = [torch.empty(sh, dtype=torch.int64, device=dev)
           for sh in ((G, A), (G, K, A), (G, K, A), (G, K, K2, A), (G, K, K2, Vs, A), (G, K, K2, Vs),
                      (G, K, Id, A), (G, K, Id) if K2w == 1 else (G, K, Id, K2w))]
    nval = torch.empty((G, K, K2), dtype=torch.int32, device=dev)
    id_n = torch.empty((G, K), dtype=torch.int32, device=dev)
    flags = torch.empty(G, dtype=torch.int32, device=dev)
    b = _abi.MapNestedBatch()
    b.G, b.R, b.K, b.K2, b.V, b.A = G, R, K, K2, V, A
    b.clock, b.ec, b.ic, b.iec, b.ivc, b.ivv = (t.data_ptr() for t in (c, e, i, ie, vc, vv))
    b.id_off, b.Di = id_off.data_ptr(), Di
    if Di > 0:
        b.id_clock, b.id_keys = id_clock.data_ptr(), id_keys.data_ptr()
    ob = _abi.MapNestedOut()
    ob.clock, ob.ec, ob.ic, ob.iec, ob.ivc, ob.ivv, ob.id_clock, ob.id_keys = (t.data_ptr() for t in out)
    ob.nval, ob.id_n, ob.flags, ob.Id, ob.Vs = nval.data_ptr(), id_n.data_ptr(), flags.data_ptr(), Id, Vs
    keep = keys_out = None
    off_arr = None
    if def_off is not None:
        off = np.asarray(def_off, dtype=np.uint64)
        if off.shape != (G + 1,):
            raise ValueError(f"map.nested_lub_many: def_off must have G+1 = {G + 1} entries")
        D = int(off[-1])
        if D > 0:
            for t, nm, shape in ((def_clock, "def_clock", (D, A)), (def_keys, "def_keys", (D, Kw)),
                                 (def_row, "def_row", (D,))):
                if t is None or not t.is_contiguous() or tuple(t.shape) != shape:
                    raise ValueError(f"map.nested_lub_many: {nm} must be a contiguous {shape} tensor")
                if nm != "def_row":
                    ctx.check_tensor(t, f"map.nested_lub_many({nm})")
            if def_row.dtype not in (torch.int32, torch.uint32) or def_row.device != dev:
                raise ValueError(f"map.nested_lub_many: def_row must be an int32 tensor on {dev}")
            off_arr = (ctypes.c_size_t * (G + 1))(*[int(x) for x in off])
            b.def_off = ctypes.cast(off_arr, ctypes.POINTER(ctypes.c_size_t))
            b.def_row, b.def_clock, b.def_keys = def_row.data_ptr(), def_clock.data_ptr(), def_keys.data_ptr()
            keep = torch.empty(D, dtype=torch.uint8, device=dev)
            keys_out = torch.empty((D, Kw), dtype=torch.int64, device=dev)
            ob.def_keep, ob.def_keys = keep.data_ptr(), keys_out.data_ptr()
    if _key_shard is None:
        ctx.call("crdt_map_nested_lub_many", ctypes.byref(b), ctypes.byref(ob))
    else:  # (shard.map_nested_lub_many_sharded)
        ctx.call("crdt_map_nested_lub_many_sharded", ctypes.byref(b), int(_key_shard[0]), int(_key_shard[1]),
                 ctypes.byref(ob))
    if check:
        f = 0
        for x in flags.cpu().numpy().tolist():
            f |= int(x)
        if f & 2:
            raise ValueError("map.nested_lub_many: def_row not non-decreasing per group or >= R")
        if f & 32:
            raise ValueError("map.nested_lub_many: id_off invalid (must start at 0, be non-decreasing and end at "
                             "id_clock.shape[0])")
        if f & 8:
            raise RuntimeError("map.nested_lub_many: more live removes named one key than the deep pass holds")
        if f & 16:
            raise RuntimeError(f"map.nested_lub_many: more than id_cap = {Id} deferred removes in one key's inner "
                               "Map (id_cap='auto' always fits)")
        if f & 64:
            raise RuntimeError(f"map.nested_lub_many: more than v_cap = {Vs} values on one inner key")
    oclk, oec, oic, oiec, oivc, oivv, oidc, oidk = out
    if squeeze:
        oclk, oec, oic, oiec, oivc, oivv, nval, id_n, oidc, oidk = (
            oclk[0], oec[0], oic[0], oiec[0], oivc[0], oivv[0], nval[0], id_n[0], oidc[0], oidk[0])
    return MapNestedLub(oclk, oec, oic, oiec, oivc, oivv, nval, id_n, oidc, oidk, flags, keep, keys_out)


# ---- Causal::forget of value-typed Map states (round 5) --------------------------------------------
def counter_forget_batch(clock: torch.Tensor, ec: torch.Tensor, val: torch.Tensor, y: torch.Tensor,
                         def_clock: Optional[torch.Tensor] = None, def_state: Optional[torch.Tensor] = None,
                         ctx: Optional[Context] = None) -> Optional[torch.Tensor]:
    """Causal::forget of N Map<K, GCounter / PNCounter> states in place (map.rs:85-114 with
    gcounter.rs:51-53 / pncounter.rs:78-81; crdt_map_counter_forget_batch): clock (N, A), ec (N, K, A),
    val (N, K, W, A) — the counter_lub_many output layout —, y (A,) or (N, A); deferred as for
    forget_batch.  Returns def_keep or None."""
    ctx = ctx or Context.default(clock.device.index)
    for t, nm in ((clock, "clock"), (ec, "ec"), (val, "val")):
        ctx.check_tensor(t, f"map.counter_forget_batch({nm})")
    if clock.dim() != 2 or ec.dim() != 3 or val.dim() != 4:
        raise ValueError("map.counter_forget_batch: clock (N,A), ec (N,K,A), val (N,K,W,A) expected")
    N, A = clock.shape
    K, W = val.shape[1], val.shape[2]
    if (tuple(ec.shape) != (N, K, A) or tuple(val.shape) != (N, K, W, A) or W not in (1, 2)
            or clock.stride(1) != 1 or ec.stride(2) != 1 or ec.stride(1) != A or val.stride(3) != 1
            or val.stride(2) != A or val.stride(1) != W * A):
        raise ValueError("map.counter_forget_batch: per-state blocks must be packed (K, A) / (K, W, A), W = 1 or 2")
    y, ys = _forget_clock(ctx, y, N, A, "map.counter_forget_batch(y)")
    dp, sp, D, keep = _forget_deferred(ctx, def_clock, def_state, N, A, "map.counter_forget_batch(def_clock)")
    st = _abi.MapCounterStates()
    st.N, st.K, st.A, st.W = N, K, A, W
    st.clock, st.clock_stride = clock.data_ptr(), clock.stride(0)
    st.ec, st.ec_stride = ec.data_ptr(), ec.stride(0)
    st.val, st.val_stride = val.data_ptr(), val.stride(0)
    ctx.call("crdt_map_counter_forget_batch", ctypes.byref(st), y.data_ptr(), ys, dp, sp, D,
             keep.data_ptr() if keep is not None else None)
    return keep


def _vd_slots(st, N: int, K: int, M: int, A: int, what: str) -> int:
    """The nested slots per key Vd of a Map<K, Orswot> state layout: vd_clock (N, K, Vd, A), vd_mem
    (N, K, Vd) or (N, K, Vd, Mw) past M = 64, vd_n (N, K) int32 (crdt_map_orswot_states.Vd)."""
    Vd = st.vd_clock.shape[2] if st.vd_clock.dim() == 4 else -1
    Mw = (M + 63) // 64 if M > 64 else 1
    vm = (N, K, Vd) if Mw == 1 else (N, K, Vd, Mw)
    if (Vd < VD_CAP or tuple(st.vd_clock.shape) != (N, K, Vd, A) or tuple(st.vd_mem.shape) != vm
            or tuple(st.vd_n.shape) != (N, K)):
        raise ValueError(f"{what}: vd_clock (N, K, Vd, A), vd_mem {'(N, K, Vd)' if Mw == 1 else '(N, K, Vd, Mw)'} "
                         f"with Vd >= {VD_CAP} and vd_n (N, K) expected")
    return Vd


def orswot_forget_batch(res: "MapOrswotLub", y: torch.Tensor, def_clock: Optional[torch.Tensor] = None,
                        def_state: Optional[torch.Tensor] = None,
                        ctx: Optional[Context] = None) -> Optional[torch.Tensor]:
    """Causal::forget of N Map<K, Orswot> states in place (map.rs:85-114 with orswot.rs:150-183;
    crdt_map_orswot_forget_batch): `res` an orswot_lub_many result with G = N states (its tensors are
    updated: clock, ec, oc, ent, vd_n, vd_clock, vd_mem), y (A,) or (N, A); the Map-level deferred rm
    clocks as for forget_batch.  Returns def_keep or None."""
    clock, ec, oc, ent = res.clock, res.ec, res.oc, res.ent
    if clock.dim() != 2:
        raise ValueError("map.orswot_forget_batch: a grouped result (clock (N, A)) expected")
    ctx = ctx or Context.default(clock.device.index)
    N, A = clock.shape
    K, M = ent.shape[1], ent.shape[2]
    for t in (clock, ec, oc, ent, res.vd_n, res.vd_clock, res.vd_mem):
        if not t.is_contiguous():
            raise ValueError("map.orswot_forget_batch: the result's tensors must be contiguous")
    Vd = _vd_slots(res, N, K, M, A, "map.orswot_forget_batch")
    y, ys = _forget_clock(ctx, y, N, A, "map.orswot_forget_batch(y)")
    dp, sp, D, keep = _forget_deferred(ctx, def_clock, def_state, N, A, "map.orswot_forget_batch(def_clock)")
    st = _abi.MapOrswotStates()
    st.N, st.K, st.M, st.A, st.Vd = N, K, M, A, Vd
    st.clock, st.ec, st.oc, st.ent = clock.data_ptr(), ec.data_ptr(), oc.data_ptr(), ent.data_ptr()
    st.vd_n, st.vd_clock, st.vd_mem = res.vd_n.data_ptr(), res.vd_clock.data_ptr(), res.vd_mem.data_ptr()
    ctx.call("crdt_map_orswot_forget_batch", ctypes.byref(st), y.data_ptr(), ys, dp, sp, D,
             keep.data_ptr() if keep is not None else None)
    return keep


# ---- CmRDT::apply of Map<K, GCounter / PNCounter> (round 5) ---------------------------------------
class MapCounterOpBatch(NamedTuple):
    """Device op streams (crdt_map_counter_ops): state s applies ops [op_off[s], op_off[s+1]) in order."""
    op_off: torch.Tensor    # (N+1,) int64
    kind: torch.Tensor      # (n_ops,) uint8: 0 = Op::Up, 1 = Op::Rm
    actor: torch.Tensor     # (n_ops,) int32   Up: the Map's dot
    counter: torch.Tensor   # (n_ops,) int64
    key: torch.Tensor       # (n_ops,) int32
    vactor: torch.Tensor    # (n_ops,) int32   Up: the counter's dot
    vcounter: torch.Tensor  # (n_ops,) int64
    vdir: torch.Tensor      # (n_ops,) uint8   0 = P, 1 = N
    clk_row: torch.Tensor   # (n_ops,) int32   Rm: row of clk_pool
    clk_pool: torch.Tensor  # (n_clk, A) int64
    key_off: torch.Tensor   # (n_ops+1,) int64 Rm keysets
    keys: torch.Tensor      # (n_keys,) int32


def encode_counter_ops(streams, A: int, device) -> MapCounterOpBatch:
    """Host ingest of per-state op streams: ("up", actor, counter, key, vactor, vcounter, dir) for
    Op::Up { dot, key, op } with the counter's op a Dot (dir 0; PNCounter: dir 1 = Neg), or
    ("rm", clock, keys) for Op::Rm { clock, keyset } (clock: mapping actor -> counter or a row)."""
    def row(clk):
        r = np.zeros(A, dtype=np.uint64)
        if hasattr(clk, "items"):
            for a, c in clk.items():
                r[int(a)] = np.uint64(c)
        else:
            r[:] = np.asarray(clk, dtype=np.uint64)
        return r

    op_off, kind, actor, counter, key, vactor, vcounter, vdir = [0], [], [], [], [], [], [], []
    clk_row, key_off, keys, pool = [], [0], [], []
    for ops in streams:
        for op in ops:
            if op[0] == "up":
                _, a, c, k, va, vc, d = op
                kind.append(0)
                actor.append(int(a)); counter.append(int(c)); key.append(int(k))  # noqa: E702
                vactor.append(int(va)); vcounter.append(int(vc)); vdir.append(int(d))  # noqa: E702
                clk_row.append(0)
            else:
                _, rc, ks = op
                kind.append(1)
                actor.append(0); counter.append(0); key.append(0)  # noqa: E702
                vactor.append(0); vcounter.append(0); vdir.append(0)  # noqa: E702
                clk_row.append(len(pool))
                pool.append(row(rc))
                keys.extend(int(x) for x in ks)
            key_off.append(len(keys))
        op_off.append(len(kind))
    i64 = lambda x: torch.tensor(np.asarray(x, dtype=np.uint64).view(np.int64), device=device)  # noqa: E731
    pool_t = (torch.from_numpy(np.stack(pool).view(np.int64)).to(device) if pool
              else torch.zeros((1, A), dtype=torch.int64, device=device))
    return MapCounterOpBatch(
        i64(op_off), torch.tensor(kind, dtype=torch.uint8, device=device),
        torch.tensor(actor, dtype=torch.int32, device=device), i64(counter),
        torch.tensor(key, dtype=torch.int32, device=device), torch.tensor(vactor, dtype=torch.int32, device=device),
        i64(vcounter), torch.tensor(vdir, dtype=torch.uint8, device=device),
        torch.tensor(clk_row, dtype=torch.int32, device=device), pool_t, i64(key_off),
        torch.tensor(keys if keys else [0], dtype=torch.int32, device=device))


_I64 = (torch.int64,)
_I32 = (torch.int32,)
_U8 = (torch.uint8,)


def _check_op_fields(ctx: Context, ops, n: int, fields, what: str) -> None:
    """Every per-op field of an op batch: shape (n,), the dtype the header states, on the ctx's device,
    contiguous.  The header-batched apply kernels load each field for every op index below n_ops, so a
    shorter, wrongly typed or host-resident field would be read out of bounds on the device."""
    for nm, dts in fields:
        t = getattr(ops, nm)
        ctx.check_tensor(t, f"{what}({nm})", dts)
        if tuple(t.shape) != (n,) or not t.is_contiguous():
            raise ValueError(f"{what}: {nm} must be a contiguous ({n},) tensor, got {tuple(t.shape)}")


def _check_op_pools(ctx: Context, ops, pools, what: str) -> None:
    """The pooled arrays (offsets, key / member lists, clock rows): dtype, device, contiguity; their
    lengths are what the kernels bound every offset by."""
    for nm, dts in pools:
        t = getattr(ops, nm)
        ctx.check_tensor(t, f"{what}({nm})", dts)
        if not t.is_contiguous():
            raise ValueError(f"{what}: {nm} must be contiguous")


def counter_apply_batch(clock: torch.Tensor, ec: torch.Tensor, val: torch.Tensor, def_clock: torch.Tensor,
                        def_keys: torch.Tensor, def_count: torch.Tensor, ops: MapCounterOpBatch,
                        ctx: Optional[Context] = None) -> torch.Tensor:
    """Apply every state's op stream in place (crdt_map_counter_apply_batch): clock (N, A), ec (N, K, A),
    val (N, K, W, A), deferred slots def_clock (N, Dcap, A) / def_keys (N, Dcap, ceil(K/64)) / def_count
    (N,) int32.  Returns the per-state status (N,) int32 (include/crdt_gpu.h)."""
    ctx = ctx or Context.default(clock.device.index)
    for t_, nm in ((clock, "clock"), (ec, "ec"), (val, "val"), (def_clock, "def_clock"), (def_keys, "def_keys")):
        ctx.check_tensor(t_, f"map.counter_apply_batch({nm})")
    N, A = clock.shape
    K, W = val.shape[1], val.shape[2]
    Kw = (K + 63) // 64
    Dcap = def_clock.shape[1]
    if (tuple(ec.shape) != (N, K, A) or tuple(val.shape) != (N, K, W, A) or not clock.is_contiguous()
            or not ec.is_contiguous() or not val.is_contiguous()):
        raise ValueError("map.counter_apply_batch: contiguous clock (N,A), ec (N,K,A), val (N,K,W,A) expected")
    if (tuple(def_clock.shape) != (N, Dcap, A) or tuple(def_keys.shape) != (N, Dcap, Kw)
            or not def_clock.is_contiguous() or not def_keys.is_contiguous() or tuple(def_count.shape) != (N,)
            or def_count.dtype != torch.int32):
        raise ValueError("map.counter_apply_batch: deferred slots (N, Dcap, A) / (N, Dcap, Kw) / (N,) int32 expected")
    n = ops.kind.shape[0]
    if ops.op_off.shape[0] != N + 1 or ops.key_off.shape[0] != n + 1 or ops.clk_pool.shape[1] != A:
        raise ValueError("map.counter_apply_batch: op_off (N+1), key_off (n_ops+1), clk_pool (n, A) expected")
    what = "map.counter_apply_batch"
    _check_op_fields(ctx, ops, n, (("kind", _U8), ("actor", _I32), ("counter", _I64), ("key", _I32),
                                   ("vactor", _I32), ("vcounter", _I64), ("vdir", _U8), ("clk_row", _I32)), what)
    _check_op_pools(ctx, ops, (("op_off", _I64), ("key_off", _I64), ("keys", _I32), ("clk_pool", _I64)), what)
    st = _abi.MapCounterStates()
    st.N, st.K, st.A, st.W = N, K, A, W
    st.clock, st.clock_stride, st.ec, st.ec_stride = clock.data_ptr(), A, ec.data_ptr(), K * A
    st.val, st.val_stride = val.data_ptr(), K * W * A
    o = _abi.MapCounterOps()
    o.n_ops, o.op_off, o.kind = n, ops.op_off.data_ptr(), ops.kind.data_ptr()
    o.actor, o.counter, o.key = ops.actor.data_ptr(), ops.counter.data_ptr(), ops.key.data_ptr()
    o.vactor, o.vcounter, o.vdir = ops.vactor.data_ptr(), ops.vcounter.data_ptr(), ops.vdir.data_ptr()
    o.clk_row, o.clk_pool, o.n_clk_rows = ops.clk_row.data_ptr(), ops.clk_pool.data_ptr(), ops.clk_pool.shape[0]
    # the pool lengths, not the (untrusted) last offsets: the kernel flags an offset past them (status bit 1)
    o.key_off, o.keys, o.n_keys = ops.key_off.data_ptr(), ops.keys.data_ptr(), ops.keys.shape[0]
    status = torch.empty(N, dtype=torch.int32, device=clock.device)
    ctx.call("crdt_map_counter_apply_batch", ctypes.byref(st), def_clock.data_ptr(), def_keys.data_ptr(),
             def_count.data_ptr(), Dcap, ctypes.byref(o), status.data_ptr())
    return status


# ---- CmRDT::apply of Map<K, Orswot> (round 5) -------------------------------------------------------
class MapOrswotOpBatch(NamedTuple):
    """Device op streams (crdt_map_orswot_ops)."""
    op_off: torch.Tensor    # (N+1,) int64
    kind: torch.Tensor      # (n_ops,) uint8: 0 = Map Op::Up, 1 = Map Op::Rm
    actor: torch.Tensor     # (n_ops,) int32   Up: the Map's dot
    counter: torch.Tensor   # (n_ops,) int64
    key: torch.Tensor       # (n_ops,) int32
    vkind: torch.Tensor     # (n_ops,) uint8   Up: 0 = Orswot Add, 1 = Orswot Rm
    vactor: torch.Tensor    # (n_ops,) int32   Add: the Orswot's dot
    vcounter: torch.Tensor  # (n_ops,) int64
    clk_row: torch.Tensor   # (n_ops,) int32   Orswot Rm / Map Rm clock row
    clk_pool: torch.Tensor  # (n_clk, A) int64
    key_off: torch.Tensor   # (n_ops+1,) int64 Map Rm keysets
    keys: torch.Tensor      # (n_keys,) int32
    mem_off: torch.Tensor   # (n_ops+1,) int64 the Orswot op's members
    mems: torch.Tensor      # (n_mems,) int32


def encode_orswot_map_ops(streams, A: int, device) -> MapOrswotOpBatch:
    """Host ingest of per-state op streams: ("add", actor, counter, key, vactor, vcounter, members),
    ("orm", actor, counter, key, clock, members) for Map Op::Up with an Orswot Add / Rm, or ("rm",
    clock, keys) for Map Op::Rm (clocks: mapping actor -> counter or a row)."""
    def row(clk):
        r = np.zeros(A, dtype=np.uint64)
        if hasattr(clk, "items"):
            for a, c in clk.items():
                r[int(a)] = np.uint64(c)
        else:
            r[:] = np.asarray(clk, dtype=np.uint64)
        return r

    f = {n: [] for n in ("kind", "actor", "counter", "key", "vkind", "vactor", "vcounter", "clk_row")}
    op_off, key_off, keys, mem_off, mems, pool = [0], [0], [], [0], [], []
    for ops in streams:
        for op in ops:
            vals = dict(kind=0, actor=0, counter=0, key=0, vkind=0, vactor=0, vcounter=0, clk_row=0)
            if op[0] == "add":
                _, a, c, k, va, vc, ms = op
                vals.update(actor=a, counter=c, key=k, vactor=va, vcounter=vc)
                mems.extend(int(x) for x in ms)
            elif op[0] == "orm":
                _, a, c, k, rc, ms = op
                vals.update(actor=a, counter=c, key=k, vkind=1, clk_row=len(pool))
                pool.append(row(rc))
                mems.extend(int(x) for x in ms)
            else:
                _, rc, ks = op
                vals.update(kind=1, clk_row=len(pool))
                pool.append(row(rc))
                keys.extend(int(x) for x in ks)
            for n, v in vals.items():
                f[n].append(int(v))
            key_off.append(len(keys))
            mem_off.append(len(mems))
        op_off.append(len(f["kind"]))
    i64 = lambda x: torch.tensor(np.asarray(x, dtype=np.uint64).view(np.int64), device=device)  # noqa: E731
    i32 = lambda x: torch.tensor(x if x else [0], dtype=torch.int32, device=device)  # noqa: E731
    u8 = lambda x: torch.tensor(x, dtype=torch.uint8, device=device)  # noqa: E731
    pool_t = (torch.from_numpy(np.stack(pool).view(np.int64)).to(device) if pool
              else torch.zeros((1, A), dtype=torch.int64, device=device))
    return MapOrswotOpBatch(i64(op_off), u8(f["kind"]), i32(f["actor"]), i64(f["counter"]), i32(f["key"]),
                            u8(f["vkind"]), i32(f["vactor"]), i64(f["vcounter"]), i32(f["clk_row"]), pool_t,
                            i64(key_off), i32(keys), i64(mem_off), i32(mems))


def orswot_apply_batch(res: "MapOrswotLub", def_clock: torch.Tensor, def_keys: torch.Tensor,
                       def_count: torch.Tensor, ops: MapOrswotOpBatch, ctx: Optional[Context] = None) -> torch.Tensor:
    """Apply every state's op stream in place (crdt_map_orswot_apply_batch): `res` an orswot_lub_many
    result with G = N states (its tensors are updated), the Map's deferred slots def_clock (N, Dcap, A)
    / def_keys (N, Dcap, ceil(K/64)) / def_count (N,) int32.  Returns the per-state status (N,) int32."""
    clock, ec, oc, ent = res.clock, res.ec, res.oc, res.ent
    if clock.dim() != 2:
        raise ValueError("map.orswot_apply_batch: a grouped result (clock (N, A)) expected")
    ctx = ctx or Context.default(clock.device.index)
    N, A = clock.shape
    K, M = ent.shape[1], ent.shape[2]
    Kw = (K + 63) // 64
    Dcap = def_clock.shape[1]
    for t_ in (clock, ec, oc, ent, res.vd_n, res.vd_clock, res.vd_mem, def_clock, def_keys):
        if not t_.is_contiguous():
            raise ValueError("map.orswot_apply_batch: contiguous tensors expected")
    if (tuple(def_clock.shape) != (N, Dcap, A) or tuple(def_keys.shape) != (N, Dcap, Kw)
            or tuple(def_count.shape) != (N,) or def_count.dtype != torch.int32):
        raise ValueError("map.orswot_apply_batch: deferred slots (N, Dcap, A) / (N, Dcap, Kw) / (N,) int32 expected")
    n = ops.kind.shape[0]
    if (ops.op_off.shape[0] != N + 1 or ops.key_off.shape[0] != n + 1 or ops.mem_off.shape[0] != n + 1
            or ops.clk_pool.shape[1] != A):
        raise ValueError("map.orswot_apply_batch: op_off (N+1), key_off / mem_off (n_ops+1), clk_pool (n, A) expected")
    what = "map.orswot_apply_batch"
    _check_op_fields(ctx, ops, n, (("kind", _U8), ("actor", _I32), ("counter", _I64), ("key", _I32),
                                   ("vkind", _U8), ("vactor", _I32), ("vcounter", _I64), ("clk_row", _I32)), what)
    _check_op_pools(ctx, ops, (("op_off", _I64), ("key_off", _I64), ("keys", _I32), ("mem_off", _I64),
                               ("mems", _I32), ("clk_pool", _I64)), what)
    st = _abi.MapOrswotStates()
    st.N, st.K, st.M, st.A = N, K, M, A
    st.Vd = _vd_slots(res, N, K, M, A, what)
    st.clock, st.ec, st.oc, st.ent = clock.data_ptr(), ec.data_ptr(), oc.data_ptr(), ent.data_ptr()
    st.vd_n, st.vd_clock, st.vd_mem = res.vd_n.data_ptr(), res.vd_clock.data_ptr(), res.vd_mem.data_ptr()
    o = _abi.MapOrswotOps()
    o.n_ops, o.op_off, o.kind = n, ops.op_off.data_ptr(), ops.kind.data_ptr()
    o.actor, o.counter, o.key = ops.actor.data_ptr(), ops.counter.data_ptr(), ops.key.data_ptr()
    o.vkind, o.vactor, o.vcounter = ops.vkind.data_ptr(), ops.vactor.data_ptr(), ops.vcounter.data_ptr()
    o.clk_row, o.clk_pool, o.n_clk_rows = ops.clk_row.data_ptr(), ops.clk_pool.data_ptr(), ops.clk_pool.shape[0]
    # the pool lengths, not the (untrusted) last offsets: the kernel flags an offset past them (status bit 1)
    o.key_off, o.keys, o.n_keys = ops.key_off.data_ptr(), ops.keys.data_ptr(), ops.keys.shape[0]
    o.mem_off, o.mems, o.n_mems = ops.mem_off.data_ptr(), ops.mems.data_ptr(), ops.mems.shape[0]
    status = torch.empty(N, dtype=torch.int32, device=clock.device)
    ctx.call("crdt_map_orswot_apply_batch", ctypes.byref(st), def_clock.data_ptr(), def_keys.data_ptr(),
             def_count.data_ptr(), Dcap, ctypes.byref(o), status.data_ptr())
    return status


# ---- CmRDT::apply and Causal::forget of Map<K, Map<K2, MVReg>> (round 5) ----------------------------
class MapNestedOpBatch(NamedTuple):
    """Device op streams (crdt_map_nested_ops): state s applies ops [op_off[s], op_off[s+1]) in order."""
    op_off: torch.Tensor    # (N+1,) int64
    kind: torch.Tensor      # (n_ops,) uint8: 0 = Op::Up, 1 = Op::Rm
    actor: torch.Tensor     # (n_ops,) int32   Up: the outer dot
    counter: torch.Tensor   # (n_ops,) int64
    key: torch.Tensor       # (n_ops,) int32
    ikind: torch.Tensor     # (n_ops,) uint8   Up: 0 inner Up (MVReg Put), 1 inner Rm
    iactor: torch.Tensor    # (n_ops,) int32   inner Up: its dot
    icounter: torch.Tensor  # (n_ops,) int64
    ikey: torch.Tensor      # (n_ops,) int32
    val: torch.Tensor       # (n_ops,) int64   inner Up: the Put's value
    ikeys: torch.Tensor     # (n_ops,) int64   inner Rm: inner-key mask ((n_ops, K2w) words past K2 = 64)
    clk_row: torch.Tensor   # (n_ops,) int32   the Put clock / an rm clock
    clk_pool: torch.Tensor  # (n_clk, A) int64
    key_off: torch.Tensor   # (n_ops+1,) int64 outer Rm keysets
    keys: torch.Tensor      # (n_keys,) int32


def encode_nested_ops(streams, A: int, device, K2: int = 64) -> MapNestedOpBatch:
    """Host ingest of per-state op streams: ("put", actor, counter, key, iactor, icounter, ikey, clock, val)
    for Op::Up { dot, key, op: inner Op::Up { dot, key, op: Put { clock, val } } }, ("irm", actor,
    counter, key, clock, ikeys) for Op::Up with an inner Op::Rm { clock, keyset }, ("rm", clock, keys)
    for Op::Rm (clocks: mapping actor -> counter or a row).  K2 > 64 (up to 256): the inner key sets
    are (n_ops, ceil(K2/64)) mask words, the layout crdt_map_nested_apply_batch reads for such states."""
    K2w = (K2 + 63) // 64 if K2 > 64 else 1
    def row(clk):
        r = np.zeros(A, dtype=np.uint64)
        if hasattr(clk, "items"):
            for a, c in clk.items():
                r[int(a)] = np.uint64(c)
        else:
            r[:] = np.asarray(clk, dtype=np.uint64)
        return r

    names = ("kind", "actor", "counter", "key", "ikind", "iactor", "icounter", "ikey", "val", "ikeys", "clk_row")
    f = {n: [] for n in names}
    op_off, key_off, keys, pool = [0], [0], [], []
    for ops in streams:
        for op in ops:
            v = dict.fromkeys(names, 0)
            if op[0] == "put":
                _, a, c, k, ia, ic, j, rc, x = op
                v.update(actor=a, counter=c, key=k, iactor=ia, icounter=ic, ikey=j, val=x, clk_row=len(pool))
            elif op[0] == "irm":
                _, a, c, k, rc, js = op
                v.update(actor=a, counter=c, key=k, ikind=1, ikeys=sum(1 << int(j) for j in set(js)), clk_row=len(pool))
                if v["ikeys"] >> (64 * K2w):
                    raise ValueError(f"encode_nested_ops: an inner key past {64 * K2w} (K2 = {K2})")
            else:
                _, rc, ks = op
                v.update(kind=1, clk_row=len(pool))
                keys.extend(int(x) for x in ks)
            pool.append(row(rc))
            for n, x in v.items():
                if n == "ikeys" and K2w > 1:
                    f[n].extend((int(x) >> (64 * w)) & 0xFFFFFFFFFFFFFFFF for w in range(K2w))
                else:
                    f[n].append(int(x))
            key_off.append(len(keys))
        op_off.append(len(f["kind"]))
    i64 = lambda x: torch.tensor(np.asarray(x, dtype=np.uint64).view(np.int64), device=device)  # noqa: E731
    i32 = lambda x: torch.tensor(x if x else [0], dtype=torch.int32, device=device)  # noqa: E731
    u8 = lambda x: torch.tensor(x, dtype=torch.uint8, device=device)  # noqa: E731
    pool_t = (torch.from_numpy(np.stack(pool).view(np.int64)).to(device) if pool
              else torch.zeros((1, A), dtype=torch.int64, device=device))
    ikeys = i64(f["ikeys"])
    if K2w > 1:
        ikeys = ikeys.reshape(-1, K2w)
    return MapNestedOpBatch(i64(op_off), u8(f["kind"]), i32(f["actor"]), i64(f["counter"]), i32(f["key"]),
                            u8(f["ikind"]), i32(f["iactor"]), i64(f["icounter"]), i32(f["ikey"]), i64(f["val"]),
                            ikeys, i32(f["clk_row"]), pool_t, i64(key_off), i32(keys))


def _nested_states(res, what):
    clock = res.clock
    if clock.dim() != 2:
        raise ValueError(f"{what}: a grouped result (clock (N, A)) expected")
    N, A = clock.shape
    K, K2 = res.iec.shape[1], res.iec.shape[2]
    K2w = (K2 + 63) // 64 if K2 > 64 else 1  # inner key sets: K2w mask words past K2 = 64
    Id = res.id_clock.shape[2] if res.id_clock.dim() == 4 else -1  # inner deferred slots per key
    if Id < NM_ID:
        raise ValueError(f"{what}: id_clock (N, K, Id, A) with Id >= {NM_ID} expected")
    Vs = res.ivc.shape[3] if res.ivc.dim() == 5 else -1  # MVReg slots per inner key
    if not NM_VS <= Vs <= 64:
        raise ValueError(f"{what}: ivc (N, K, K2, Vs, A) with Vs in {NM_VS}..64 expected")
    shapes = dict(ec=(N, K, A), ic=(N, K, A), iec=(N, K, K2, A), ivc=(N, K, K2, Vs, A), ivv=(N, K, K2, Vs),
                  nval=(N, K, K2), id_n=(N, K), id_clock=(N, K, Id, A),
                  id_keys=(N, K, Id) if K2w == 1 else (N, K, Id, K2w))
    for nm, shp in shapes.items():
        t = getattr(res, nm)
        if tuple(t.shape) != shp or not t.is_contiguous():
            raise ValueError(f"{what}: {nm} must be a contiguous {shp} tensor")
    if not clock.is_contiguous():
        raise ValueError(f"{what}: clock must be contiguous")
    st = _abi.MapNestedStates()
    st.N, st.K, st.K2, st.A, st.Id, st.Vs = N, K, K2, A, Id, Vs
    for nm in ("clock", "ec", "ic", "iec", "ivc", "ivv", "nval", "id_n", "id_clock", "id_keys"):
        setattr(st, nm, getattr(res, nm).data_ptr())
    return st, N, K, A


def nested_apply_batch(res: "MapNestedLub", def_clock: torch.Tensor, def_keys: torch.Tensor,
                       def_count: torch.Tensor, ops: MapNestedOpBatch, ctx: Optional[Context] = None) -> torch.Tensor:
    """Apply every state's op stream in place (crdt_map_nested_apply_batch): `res` a nested_lub_many
    result with G = N states (its tensors are updated), the outer deferred slots def_clock (N, Dcap, A)
    / def_keys (N, Dcap, ceil(K/64)) / def_count (N,) int32.  Returns the per-state status (N,) int32.
    K2 > 64 (up to 256): id_keys (N, K, 16, K2w) and ops.ikeys (n_ops, K2w) mask words
    (encode_nested_ops(..., K2=K2))."""
    st, N, K, A = _nested_states(res, "map.nested_apply_batch")
    ctx = ctx or Context.default(res.clock.device.index)
    Kw = (K + 63) // 64
    Dcap = def_clock.shape[1]
    if (tuple(def_clock.shape) != (N, Dcap, A) or tuple(def_keys.shape) != (N, Dcap, Kw)
            or tuple(def_count.shape) != (N,) or def_count.dtype != torch.int32
            or not def_clock.is_contiguous() or not def_keys.is_contiguous()):
        raise ValueError("map.nested_apply_batch: deferred slots (N, Dcap, A) / (N, Dcap, Kw) / (N,) int32 expected")
    n = ops.kind.shape[0]
    if ops.op_off.shape[0] != N + 1 or ops.key_off.shape[0] != n + 1 or ops.clk_pool.shape[1] != A:
        raise ValueError("map.nested_apply_batch: op_off (N+1), key_off (n_ops+1), clk_pool (n, A) expected")
    what = "map.nested_apply_batch"
    _check_op_fields(ctx, ops, n, (("kind", _U8), ("actor", _I32), ("counter", _I64), ("key", _I32),
                                   ("ikind", _U8), ("iactor", _I32), ("icounter", _I64), ("ikey", _I32),
                                   ("val", _I64), ("clk_row", _I32)), what)
    _check_op_pools(ctx, ops, (("op_off", _I64), ("key_off", _I64), ("keys", _I32), ("clk_pool", _I64)), what)
    K2 = res.iec.shape[2]
    K2w = (K2 + 63) // 64 if K2 > 64 else 1
    ctx.check_tensor(ops.ikeys, f"{what}(ikeys)", _I64)
    ik_shape = (n,) if K2w == 1 else (n, K2w)
    if tuple(ops.ikeys.shape) != ik_shape or not ops.ikeys.is_contiguous():
        raise ValueError(f"{what}: ikeys must be a contiguous {ik_shape} tensor (K2 = {K2}), "
                         f"got {tuple(ops.ikeys.shape)}")
    o = _abi.MapNestedOps()
    o.n_ops, o.op_off = n, ops.op_off.data_ptr()
    for nm in ("kind", "actor", "counter", "key", "ikind", "iactor", "icounter", "ikey", "val", "ikeys", "clk_row",
               "key_off", "keys"):
        setattr(o, nm, getattr(ops, nm).data_ptr())
    o.clk_pool, o.n_clk_rows = ops.clk_pool.data_ptr(), ops.clk_pool.shape[0]
    o.n_keys = ops.keys.shape[0]
    status = torch.zeros(N, dtype=torch.int32, device=res.clock.device)
    ctx.call("crdt_map_nested_apply_batch", ctypes.byref(st), def_clock.data_ptr(), def_keys.data_ptr(),
             def_count.data_ptr(), Dcap, ctypes.byref(o), status.data_ptr())
    return status


def nested_forget_batch(res: "MapNestedLub", y: torch.Tensor, def_clock: Optional[torch.Tensor] = None,
                        def_state: Optional[torch.Tensor] = None,
                        ctx: Optional[Context] = None) -> Optional[torch.Tensor]:
    """Causal::forget of N Map<K, Map<K2, MVReg>> states in place (map.rs:85-114 at both levels,
    mvreg.rs:88-104; crdt_map_nested_forget_batch): `res` a nested_lub_many result with G = N states,
    y (A,) or (N, A); the outer deferred rm clocks as for forget_batch.  Returns def_keep or None."""
    st, N, K, A = _nested_states(res, "map.nested_forget_batch")
    ctx = ctx or Context.default(res.clock.device.index)
    y, ys = _forget_clock(ctx, y, N, A, "map.nested_forget_batch(y)")
    dp, sp, D, keep = _forget_deferred(ctx, def_clock, def_state, N, A, "map.nested_forget_batch(def_clock)")
    ctx.call("crdt_map_nested_forget_batch", ctypes.byref(st), y.data_ptr(), ys, dp, sp, D,
             keep.data_ptr() if keep is not None else None)
    return keep


# ---- Pairwise merge_batch of value-typed Map states (round 6) --------------------------------------
# self[i].merge(other[i]) for Map<K, GCounter / PNCounter>, Map<K, Orswot<M>> and Map<K, Map<K2, MVReg>>
# states in their apply layouts (wire.MapCounterFrames / MapOrswotFrames / MapNestedFrames or any
# object with those fields): crdt_map_{counter,orswot,nested}_merge_batch (csrc/vmap_merge.hip) — each
# pair one group of the exact left-fold kernel (Map::new() merged with self, then with other, R = 2),
# self's rows, nested lists and Map-level slots rewritten (the surviving removes in pool order).  Map::merge
# from an empty Map reproduces a state whose deferred removes are applied and not dominated by its
# clock — every state apply, merge, forget or ingest leaves — so this is self.merge(other) (map.rs:140-220)
# on those states.  Status bits as the header: 0 = survivors past self's Dcap (first Dcap kept), 3 = a
# fold capacity (the pair's state incomplete).
def _vm_deferred(ctx, st, N: int, A: int, Kw: int, what: str):
    Dc = st.def_clock.shape[1] if st.def_clock.dim() == 3 else 0
    if (tuple(st.def_clock.shape) != (N, Dc, A) or tuple(st.def_keys.shape) != (N, Dc, Kw)
            or not st.def_clock.is_contiguous() or not st.def_keys.is_contiguous()):
        raise ValueError(f"{what}: def_clock / def_keys must be contiguous (N, Dcap, A) / (N, Dcap, Kw)")
    if (tuple(st.def_count.shape) != (N,) or st.def_count.dtype not in (torch.int32, torch.uint32)
            or st.def_count.device != st.clock.device):
        raise ValueError(f"{what}: def_count must be an (N,) int32 tensor on the states' device")
    ctx.check_tensor(st.def_clock, f"{what}(def_clock)")
    ctx.check_tensor(st.def_keys, f"{what}(def_keys)")
    d = _abi.MapDeferred()
    d.clock, d.keys, d.count, d.Dcap = st.def_clock.data_ptr(), st.def_keys.data_ptr(), st.def_count.data_ptr(), Dc
    return d


def _same_shapes(me, other, fields, what):
    for nm in fields:
        a, b = getattr(me, nm), getattr(other, nm)
        if tuple(a.shape) != tuple(b.shape) or a.device != b.device:
            raise ValueError(f"{what}: self.{nm} {tuple(a.shape)} and other.{nm} {tuple(b.shape)} differ")
        if not a.is_contiguous() or not b.is_contiguous():
            raise ValueError(f"{what}: {nm} must be contiguous")


def _vm_call(ctx, fn, sa, sb, me, other, N, A, K, what):
    Kw = (K + 63) // 64
    da, db = _vm_deferred(ctx, me, N, A, Kw, what), _vm_deferred(ctx, other, N, A, Kw, what)
    status = torch.zeros(N, dtype=torch.int32, device=me.clock.device)
    ctx.call(fn, ctypes.byref(sa), ctypes.byref(da), ctypes.byref(sb), ctypes.byref(db), status.data_ptr())
    return status


def counter_merge_batch(me, other, ctx: Optional[Context] = None) -> torch.Tensor:
    """self[i].merge(other[i]) for N Map<K, GCounter / PNCounter> states, in place on `me`
    (crdt_map_counter_merge_batch; Map::merge map.rs:140-220 with gcounter.rs:44-54 / pncounter.rs:70-82):
    clock (N, A), ec (N, K, A), val (N, K, W, A), def_clock (N, Dcap, A), def_keys (N, Dcap, Kw),
    def_count (N,) int32 — the crdt_map_counter_states layout.  Returns status (N,) int32."""
    what = "map.counter_merge_batch"
    _same_shapes(me, other, ("clock", "ec", "val"), what)
    ctx = ctx or Context.default(me.clock.device.index)
    N, A = me.clock.shape
    K, W = me.ec.shape[1], me.val.shape[2]
    if tuple(me.ec.shape) != (N, K, A) or tuple(me.val.shape) != (N, K, W, A):
        raise ValueError(f"{what}: clock (N, A), ec (N, K, A), val (N, K, W, A) expected")
    if N == 0:
        return torch.zeros(0, dtype=torch.int32, device=me.clock.device)
    sts = []
    for st in (me, other):
        for t, nm in ((st.clock, "clock"), (st.ec, "ec"), (st.val, "val")):
            ctx.check_tensor(t, f"{what}({nm})")
        x = _abi.MapCounterStates()
        x.N, x.K, x.A, x.W = N, K, A, W
        x.clock, x.clock_stride = st.clock.data_ptr(), A
        x.ec, x.ec_stride = st.ec.data_ptr(), K * A
        x.val, x.val_stride = st.val.data_ptr(), K * W * A
        sts.append(x)
    return _vm_call(ctx, "crdt_map_counter_merge_batch", sts[0], sts[1], me, other, N, A, K, what)


def orswot_merge_batch(me, other, ctx: Optional[Context] = None) -> torch.Tensor:
    """self[i].merge(other[i]) for N Map<K, Orswot<M>> states, in place on `me`
    (crdt_map_orswot_merge_batch; Map::merge map.rs:140-220 with Orswot::merge orswot.rs:81-149 and forget
    :150-183): the crdt_map_orswot_states layout (clock, ec, oc, ent, vd_n, vd_clock, vd_mem) + the Map's
    deferred slots def_clock / def_keys / def_count.  Returns status (N,) int32."""
    what = "map.orswot_merge_batch"
    _same_shapes(me, other, ("clock", "ec", "oc", "ent", "vd_n", "vd_clock", "vd_mem"), what)
    ctx = ctx or Context.default(me.clock.device.index)
    N, A = me.clock.shape
    K, M = me.ent.shape[1], me.ent.shape[2]
    if N == 0:
        return torch.zeros(0, dtype=torch.int32, device=me.clock.device)
    sts = []
    for st in (me, other):
        for nm in ("clock", "ec", "oc", "ent", "vd_clock", "vd_mem"):
            ctx.check_tensor(getattr(st, nm), f"{what}({nm})")
        if st.vd_n.dtype != torch.int32 or tuple(st.vd_n.shape) != (N, K):
            raise ValueError(f"{what}: vd_n must be an (N, K) int32 tensor")
        x = _abi.MapOrswotStates()
        x.N, x.K, x.M, x.A = N, K, M, A
        x.Vd = _vd_slots(st, N, K, M, A, what)
        x.clock, x.ec, x.oc, x.ent = st.clock.data_ptr(), st.ec.data_ptr(), st.oc.data_ptr(), st.ent.data_ptr()
        x.vd_n, x.vd_clock, x.vd_mem = st.vd_n.data_ptr(), st.vd_clock.data_ptr(), st.vd_mem.data_ptr()
        sts.append(x)
    return _vm_call(ctx, "crdt_map_orswot_merge_batch", sts[0], sts[1], me, other, N, A, K, what)


def nested_merge_batch(me, other, ctx: Optional[Context] = None) -> torch.Tensor:
    """self[i].merge(other[i]) for N Map<K, Map<K2, MVReg<u64>>> states, in place on `me`
    (crdt_map_nested_merge_batch; Map::merge map.rs:140-220 at both levels, MVReg::merge mvreg.rs:112-128):
    the crdt_map_nested_states layout (clock, ec, ic, iec, ivc, ivv, nval, id_n, id_clock, id_keys) + the
    outer deferred slots def_clock / def_keys / def_count.  Returns status (N,) int32."""
    what = "map.nested_merge_batch"
    _same_shapes(me, other, ("clock", "ec", "ic", "iec", "ivc", "ivv", "nval", "id_n", "id_clock", "id_keys"), what)
    ctx = ctx or Context.default(me.clock.device.index)
    if me.clock.shape[0] == 0:
        return torch.zeros(0, dtype=torch.int32, device=me.clock.device)
    sa, N, K, A = _nested_states(me, what)
    sb, _, _, _ = _nested_states(other, what)
    return _vm_call(ctx, "crdt_map_nested_merge_batch", sa, sb, me, other, N, A, K, what)
