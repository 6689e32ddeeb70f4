"""Replica-sharded lub across the GPUs of a node: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) or gloo (CPU tests).

Each rank folds its own contiguous replica range locally (lub_many), then ONE exchange
combines the per-rank partial states:
  - VClock / GCounter / PNCounter: all_reduce(MAX) of the (G, W) partial lub.  RCCL has no
    unsigned max on int64 tensors, so the u64 bits are biased by flipping the sign bit
    (x ^ 2^63 maps unsigned order onto signed order), reduced with signed MAX, and flipped back.
  - GSet: RCCL has no bitwise-OR reduction, so partials are all-gathered and OR-ed by the same
    lub kernel over `world` rows.
The lub is associative and commutative (README.md:37-47), so the sharded result equals the
single fold over all replicas bit for bit.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

SIGN = -(2**63)


def _bias(t: torch.Tensor) -> torch.Tensor:
    return t ^ torch.tensor(SIGN, dtype=t.dtype, device=t.device)


def _gloo(group) -> bool:
    return dist.get_backend(group) == "gloo"


def all_reduce_(t: torch.Tensor, op, group=None) -> torch.Tensor:
    """In-place all-reduce.  gloo has no device-memory collectives on ROCm, so a device tensor is
    staged through host memory there (tests run two ranks on one GPU that way; RCCL refuses two
    ranks per GPU).  RCCL ("nccl") reduces in place in HBM."""
    if t.is_cuda and _gloo(group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t


def allreduce_umax_(partial: torch.Tensor, group=None) -> torch.Tensor:
    """In-place unsigned-64 max all-reduce of an int64 tensor holding u64 bits."""
    if partial.dtype != torch.int64:
        raise TypeError("allreduce_umax_: int64 tensor holding u64 bits expected")
    b = _bias(partial)
    all_reduce_(b, dist.ReduceOp.MAX, group)
    partial.copy_(_bias(b))
    return partial


def allgather_rows(partial: torch.Tensor, group=None) -> torch.Tensor:
    """(…, W) partial -> (world, …, W) stacked in rank order."""
    world = dist.get_world_size(group)
    out = torch.empty((world,) + tuple(partial.shape), dtype=partial.dtype, device=partial.device)
    if _gloo(group):  # gloo has no all_gather_into_tensor and no device-memory collectives here
        host = torch.empty((world,) + tuple(partial.shape), dtype=partial.dtype)
        dist.all_gather(list(host.unbind(0)), partial.contiguous().cpu(), group=group)
        out.copy_(host)
    else:
        dist.all_gather_into_tensor(out, partial.contiguous(), group=group)
    return out


def lub_many_sharded(kind: str, shard: torch.Tensor, group=None,
                     local_lub: Optional[Callable[[torch.Tensor], torch.Tensor]] = None) -> torch.Tensor:
    """Global lub of the replicas held across ranks; `shard` is this rank's (R_local, W) or
    (G, R_local, W) slice.  `local_lub` defaults to the HIP kernels of `kind` (tests inject a
    checker on CPU-only hosts to exercise the exchange with gloo)."""
    if local_lub is None:
        from . import gcounter, gset, pncounter, vclock
        local_lub = {"vclock": vclock.lub_many, "gcounter": gcounter.lub_many,
                     "pncounter": pncounter.lub_many, "gset": gset.lub_many}[kind]
    partial = local_lub(shard)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return partial
    if kind in ("vclock", "gcounter", "pncounter"):
        return allreduce_umax_(partial, group)
    if kind == "gset":
        rows = allgather_rows(partial, group)  # (world, [G,] W)
        if rows.dim() == 3:
            rows = rows.transpose(0, 1)  # (G, world, W) for a grouped lub
        return local_lub(rows.contiguous())
    raise ValueError(f"lub_many_sharded: unsupported kind {kind!r}")


def shard_range(R: int, rank: int, world: int):
    """Contiguous replica range [lo, hi) of `rank` (sizes differ by at most one)."""
    base, extra = divmod(R, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


# ---- LWWReg ---------------------------------------------------------------------------------
NO_CONFLICT = 2**63 - 1  # int64 stand-in for u64::MAX in the MIN all-reduce


def lwwreg_lub_many_sharded(marker: torch.Tensor, val: torch.Tensor, base: int, group=None,
                            local=None):
    """Exact sharded LWW fold (state AND first conflicting merge) over replicas split in rank
    order: rank k holds replicas [base, base + R_k) of every group ((R_k,) or (G, R_k)).

    1. local fold of each shard; all-gather the (G,) marker/val states;
    2. rank k folds the states of ranks < k (the prefix) and re-runs its shard continuing from
       that prefix (CRDT_ACCUMULATE), which yields the conflict indices of the GLOBAL fold;
    3. MIN all-reduce of base + local index; the final state is the fold of all rank states.
    Returns (marker (G,), val (G,), first_conflict (G,) int64, -1 = none)."""
    if local is None:
        from . import lwwreg
        local = lwwreg.lub_many
    squeeze = marker.dim() == 1
    m2 = marker.reshape(1, -1) if squeeze else marker
    v2 = val.reshape(1, -1) if squeeze else val
    G = m2.shape[0]
    lm, lv, lf = local(m2, v2)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if world == 1:
        fc = torch.where(lf == -1, lf, lf + base)
        return (lm[0], lv[0], fc[0]) if squeeze else (lm, lv, fc)
    states = allgather_rows(torch.stack([lm, lv]), group)  # (world, 2, G)
    gm = states[:, 0, :].transpose(0, 1).contiguous()  # (G, world)
    gv = states[:, 1, :].transpose(0, 1).contiguous()
    if rank > 0:
        pm, pv, _ = local(gm[:, :rank].contiguous(), gv[:, :rank].contiguous())
        _, _, lf = local(m2, v2, init=(pm, pv))
    fc = torch.where(lf == -1, torch.full_like(lf, NO_CONFLICT), lf + base)
    all_reduce_(fc, dist.ReduceOp.MIN, group)
    fc = torch.where(fc == NO_CONFLICT, torch.full_like(fc, -1), fc)
    fm, fv, _ = local(gm, gv)
    return (fm[0], fv[0], fc[0]) if squeeze else (fm, fv, fc)


# ---- Orswot ---------------------------------------------------------------------------------
def orswot_lub_many_sharded(clock: torch.Tensor, entries: torch.Tensor, def_clock: torch.Tensor,
                            def_members: torch.Tensor, def_group: torch.Tensor, group=None,
                            local=None):
    """Sharded Orswot lub: rank k holds replicas of every group ((G, R_k, A) / (G, R_k, M, A))
    plus its replicas' deferred removes, pooled as rows with their group ids `def_group` (D_k,).

    The dot-store join is associative under the reference invariants, so each rank joins its
    shard WITHOUT deferred removes, the partial (clock, entries) states are all-gathered, and
    every rank re-merges the `world` partials together with ALL ranks' deferred removes (the
    forget ceiling and the survival test need the global clock).  Returns an OrswotLub."""
    if local is None:
        from . import orswot
        local = orswot.lub_many
    G, _, A = clock.shape
    M = entries.shape[2]
    part = local(clock, entries)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        pc, pe = part.clock.unsqueeze(1), part.entries.unsqueeze(1)
        dcl, dmem, dgrp = def_clock, def_members, def_group
    else:
        pc = allgather_rows(part.clock, group).transpose(0, 1).contiguous()    # (G, world, A)
        pe = allgather_rows(part.entries, group).transpose(0, 1).contiguous()  # (G, world, M, A)
        # deferred removes: sizes first, then padded rows
        n = torch.tensor([def_clock.shape[0]], dtype=torch.int64, device=clock.device)
        ns = allgather_rows(n, group).reshape(-1).tolist()
        dmax = max(1, max(ns))
        Mw = def_members.shape[1]
        pad = torch.zeros((dmax, A + Mw + 1), dtype=torch.int64, device=clock.device)
        k = def_clock.shape[0]
        if k:
            pad[:k, :A] = def_clock
            pad[:k, A:A + Mw] = def_members
            pad[:k, A + Mw] = def_group.to(torch.int64)
        allp = allgather_rows(pad, group)  # (world, dmax, A+Mw+1)
        rows = torch.cat([allp[r, :ns[r]] for r in range(world)]) if sum(ns) else pad[:0]
        dcl, dmem, dgrp = rows[:, :A], rows[:, A:A + Mw], rows[:, A + Mw]
    # pool the deferred removes by group (stable: rank order, then local order)
    if dcl.shape[0]:
        order = torch.argsort(dgrp, stable=True)
        dcl, dmem = dcl[order].contiguous(), dmem[order].contiguous()
        counts = torch.bincount(dgrp.to(torch.int64), minlength=G).tolist()
        off = [0]
        for c in counts:
            off.append(off[-1] + c)
        return local(pc, pe, def_off=off, def_clock=dcl, def_members=dmem)
    return local(pc, pe)


# ---- Map<K, MVReg> ----------------------------------------------------------------------------
def _key_bits(bitmaps: torch.Tensor) -> torch.Tensor:
    """(D, Kw) int64 key bitmaps -> (D, Kw*64) 0/1 int64."""
    sh = torch.arange(64, device=bitmaps.device, dtype=torch.int64)
    return ((bitmaps.unsqueeze(-1) >> sh) & 1).reshape(bitmaps.shape[0], -1)


def _pack_bits(bits: torch.Tensor) -> torch.Tensor:
    """(D, n) 0/1 int64 -> (D, ceil(n/64)) int64 bitmaps (distinct bits: the sum is the OR)."""
    D, n = bits.shape
    Kw = (n + 63) // 64
    pad = torch.zeros((D, Kw * 64), dtype=torch.int64, device=bits.device)
    pad[:, :n] = bits
    sh = torch.arange(64, device=bits.device, dtype=torch.int64)
    return (pad.reshape(D, Kw, 64) << sh).sum(-1)


def restrict_key_bitmaps(bitmaps: torch.Tensor, k0: int, Kk: int) -> torch.Tensor:
    """Key bitmaps over all keys -> bitmaps over keys [k0, k0+Kk) re-indexed from 0."""
    return _pack_bits(_key_bits(bitmaps)[:, k0:k0 + Kk])


def expand_key_bitmaps(bitmaps: torch.Tensor, k0: int, K: int) -> torch.Tensor:
    """Bitmaps over local keys [0, Kk) -> bitmaps over all K keys (local key i = key k0 + i)."""
    loc = _key_bits(bitmaps)
    full = torch.zeros((bitmaps.shape[0], K), dtype=torch.int64, device=bitmaps.device)
    n = min(loc.shape[1], K - k0)
    full[:, k0:k0 + n] = loc[:, :n]
    return _pack_bits(full)


def map_lub_many_sharded(clock: torch.Tensor, ec: torch.Tensor, vclk: torch.Tensor, vval: torch.Tensor,
                         k0: int, K: int, def_off=None, def_row=None, def_clock=None, def_keys=None,
                         vout: int = 4, group=None, local=None):
    """Key-sharded Map<K, MVReg> lub: rank k owns keys [k0, k0 + Kk) of every replica
    (ec (G, R, Kk, A), vclk (G, R, Kk, V, A), vval (G, R, Kk, V)) and holds every replica's map
    clock (G, R, A) and the group's whole deferred list (key bitmaps over all K keys).

    Keys are independent given the replica clocks and the deferred list (csrc/map.hip header), so
    each rank's fold of its keys is the exact left fold with no data-path collective — unlike a
    replica split, which would need the (non-associative) re-merge.  The one
    exchange is the surviving-remove output: the clock and the survival flags are the same on
    every rank; each rank's key sets cover its own keys only, so a SUM all-reduce of the
    bitmaps is their union.  Returns a MapLub whose ec / vclk / vval / nval are the rank's keys
    and whose def_keys are over all K keys."""
    if local is None:
        from . import map as cmap
        local = cmap.lub_many
    Kk = ec.shape[-2]
    kw = {}
    if def_off is not None and int(def_off[-1]) > 0:
        kw = dict(def_off=def_off, def_row=def_row, def_clock=def_clock,
                  def_keys=restrict_key_bitmaps(def_keys, k0, Kk).contiguous())
    res = local(clock, ec, vclk, vval, vout=vout, **kw)
    if res.def_keys is None:
        return res
    gk = expand_key_bitmaps(res.def_keys, k0, K)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world > 1:
        all_reduce_(gk, dist.ReduceOp.SUM, group)
    return res._replace(def_keys=gk)
