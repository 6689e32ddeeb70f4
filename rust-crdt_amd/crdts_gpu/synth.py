"""Synthetic replica states for benchmarks and parity tests, generated in HBM.

Counter-based (stateless hash) so the CPU can regenerate any sampled replica bit for bit
(oracle.synth_* restates the formulas independently).  Formulas: include/crdt_gpu.h
(crdt_synth_fill, crdt_synth_orswot).
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple, Optional

import numpy as np
import torch

from .context import Context, dptr, synth_fill  # noqa: F401

_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def orswot_clock_rows(seed: int, rows: np.ndarray, A: int, kmax: int) -> np.ndarray:
    """clock[r][a] of crdt_synth_orswot for the given global replica indices (host)."""
    rows = np.asarray(rows, dtype=np.uint64)
    idx = rows[:, None] * np.uint64(A) + np.arange(A, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        h = _mix64(np.uint64(seed) + (idx + np.uint64(1)) * _GOLD)
    return h % np.uint64(kmax + 1)


class OrswotInput(NamedTuple):
    clock: torch.Tensor      # (R, A)
    entries: torch.Tensor    # (R, M, A)
    def_off: np.ndarray      # (R+1,) per replica CSR (host)
    def_clock: torch.Tensor  # (D, A)
    def_members: torch.Tensor  # (D, Mw)


def orswot_deferred(seed: int, R: int, M: int, A: int, kmax: int, first_row: int = 0,
                    p_def: float = 0.1, max_per_replica: int = 3):
    """Host-side deferred removes for replicas [first_row, first_row+R): each replica holds one
    to `max_per_replica` removes with probability p_def, each with a "future" context
    (rm[a] = clock[a] + delta on ~10% of actors, at least one) over 1-3 members."""
    rng = np.random.default_rng(seed ^ 0xDEF0 ^ (first_row * 0x9E37))
    has = rng.random(R) < p_def
    counts = np.where(has, rng.integers(1, max_per_replica + 1, size=R), 0)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    D = int(off[-1])
    Mw = (M + 63) // 64
    rows = np.repeat(np.arange(R), counts)
    base = orswot_clock_rows(seed, rows + first_row, A, kmax) if D else np.zeros((0, A), np.uint64)
    fut = rng.random((D, A)) < 0.1
    if D:
        fut[np.arange(D), rng.integers(0, A, size=D)] = True
    delta = rng.integers(1, 4, size=(D, A)).astype(np.uint64)
    rm = np.where(fut, base + delta, base).astype(np.uint64)
    members = np.zeros((D, Mw), dtype=np.uint64)
    nm = rng.integers(1, 4, size=D)
    for d in range(D):
        for m in rng.choice(M, size=min(M, int(nm[d])), replace=False):
            members[d, m // 64] |= np.uint64(1) << np.uint64(m % 64)
    return off, rows.astype(np.uint32), rm, members


def orswot_replicas(ctx: Optional[Context], R: int, M: int, A: int, seed: int, kmax: int = 48,
                    first_row: int = 0, p_def: float = 0.1, device: Optional[torch.device] = None,
                    entries: Optional[torch.Tensor] = None, clock: Optional[torch.Tensor] = None) -> OrswotInput:
    """Generate R well-formed Orswot replicas in HBM, with deferred removes pre-applied."""
    ctx = ctx or Context.default()
    dev = device or torch.device("cuda", ctx.device)
    if clock is None:
        clock = torch.empty((R, A), dtype=torch.int64, device=dev)
    if entries is None:
        entries = torch.empty((R, M, A), dtype=torch.int64, device=dev)
    ctx.call("crdt_synth_orswot", dptr(clock), dptr(entries), R, M, A, first_row,
             ctypes.c_uint64(seed), ctypes.c_uint64(kmax))
    off, rows, rm, members = orswot_deferred(seed, R, M, A, kmax, first_row, p_def)
    D = rm.shape[0]
    dcl = torch.from_numpy(rm.view(np.int64)).to(dev)
    dmem = torch.from_numpy(members.view(np.int64)).to(dev)
    if D:
        drow = torch.from_numpy(rows.astype(np.int32)).to(dev)
        ctx.call("crdt_synth_orswot_rm", dptr(entries), M, A, D, dptr(drow), dptr(dcl), dptr(dmem))
        torch.cuda.current_stream(dev).synchronize()
    return OrswotInput(clock, entries, off, dcl, dmem)


class MapInput(NamedTuple):
    clock: torch.Tensor      # (R, A)
    ec: torch.Tensor         # (R, K, A)
    vclk: torch.Tensor       # (R, K, V, A)
    vval: torch.Tensor       # (R, K, V)
    def_off: list            # [0, D] (one group)
    def_row: torch.Tensor    # (D,) int32
    def_clock: torch.Tensor  # (D, A)
    def_keys: torch.Tensor   # (D, Kw)
    alloc: str = "torch caching allocator"  # (or "contiguous block (crdt_device_alloc)")


def map_deferred(seed: int, R: int, K: int, A: int, kmax: int, p_def: float = 0.1, first_row: int = 0):
    """Host-side deferred removes of crdt_synth_map's model (closed form in the replica index):
    replica r holds 1-2 removes with probability p_def, each by a writer w with a future
    context rm[w] = clock[r][w] + 1..4 (and a past one on a second actor) over 1-3 of w's keys.
    Returns (def_row local (D,), def_clock (D, A), def_keys (D, Kw))."""
    Kw = (K + 63) // 64
    r = np.arange(first_row, first_row + R, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = _mix64((np.uint64(seed) ^ np.uint64(0xDEF0DEF0DEF0DEF0)) + r)
    thr = int(p_def * 1000)
    nd = np.where(h % np.uint64(1000) < np.uint64(thr), np.uint64(1) + (h >> np.uint64(32)) % np.uint64(2), np.uint64(0))
    rows = np.repeat(np.arange(R), nd.astype(np.int64))
    D = rows.shape[0]
    di = np.concatenate([np.arange(int(n)) for n in nd]) if D else np.zeros(0, np.int64)
    with np.errstate(over="ignore"):
        hd = _mix64(h[rows] + np.uint64(0x9E37) * (di.astype(np.uint64) + np.uint64(1)))
    Au = np.uint64(A)
    w = (hd % Au).astype(np.int64)
    clock = map_clock_rows(seed, rows + first_row, A, kmax) if D else np.zeros((0, A), np.uint64)
    rm = np.zeros((D, A), np.uint64)
    rm[np.arange(D), w] = clock[np.arange(D), w] + np.uint64(1) + (hd >> np.uint64(8)) % np.uint64(4)
    if A > 1:
        b = ((w.astype(np.uint64) + np.uint64(1) + (hd >> np.uint64(16)) % np.uint64(A - 1)) % Au).astype(np.int64)
        rm[np.arange(D), b] = clock[np.arange(D), b] // np.uint64(2)
    keys = np.zeros((D, Kw), np.uint64)
    nk = (np.uint64(1) + (hd >> np.uint64(24)) % np.uint64(3)).astype(np.int64)
    for d in range(D):
        wk = _map_keys_of(int(w[d]), K, A)
        for i in range(int(nk[d])):
            with np.errstate(over="ignore"):
                j = int(_mix64(hd[d] + np.uint64(i + 1))) % len(wk)
            k = int(wk[j])
            keys[d, k // 64] |= np.uint64(1) << np.uint64(k % 64)
    return rows, rm, keys


def _map_keys_of(a: int, K: int, A: int) -> np.ndarray:
    if A == 1:
        return np.arange(K, dtype=np.int64)
    return np.concatenate([np.arange(a, K, A), np.arange((a - 1) % A, K, A)]).astype(np.int64)


def map_clock_rows(seed: int, rows: np.ndarray, A: int, kmax: int) -> np.ndarray:
    """clock[r][a] of crdt_synth_map for the given global replica indices (host)."""
    return orswot_clock_rows(seed, rows, A, kmax)


def map_replicas(ctx: Optional[Context], R: int, K: int, A: int, V: int, seed: int, kmax: int = 256,
                 first_row: int = 0, p_def: float = 0.1, contig: bool = False) -> MapInput:
    """Generate R well-formed Map<K, MVReg<u64>> replicas in HBM (crdt_synth_map), with their
    deferred removes (host-built, then uploaded) pre-applied.  contig: the four replica arrays as views
    of one physically contiguous device block (Context.device_empty) where one is free."""
    ctx = ctx or Context.default()
    dev = torch.device("cuda", ctx.device)
    shapes = ((R, A), (R, K, A), (R, K, V, A), (R, K, V))
    sizes = [int(np.prod(sh)) for sh in shapes]
    pad = lambda n: (n + 511) // 512 * 512  # noqa: E731  (4-KiB aligned views)
    block = ctx.device_empty((sum(pad(n) for n in sizes),)) if contig else None
    if block is not None:
        views, at = [], 0
        for sh, n in zip(shapes, sizes):
            views.append(block[at:at + n].view(sh))
            at += pad(n)
        clock, ec, vclk, vval = views
    else:
        clock, ec, vclk, vval = (torch.empty(sh, dtype=torch.int64, device=dev) for sh in shapes)
    rows, rm, keys = map_deferred(seed, R, K, A, kmax, p_def, first_row)
    D = rm.shape[0]
    off = np.searchsorted(rows, np.arange(R + 1), side="left").astype(np.int64)
    d_off = torch.from_numpy(off).to(dev)
    dcl = torch.from_numpy(np.ascontiguousarray(rm).view(np.int64)).to(dev)
    dk = torch.from_numpy(np.ascontiguousarray(keys).view(np.int64)).to(dev)
    ctx.call("crdt_synth_map", dptr(clock), dptr(ec), dptr(vclk), dptr(vval), R, K, A, V, first_row,
             ctypes.c_uint64(seed), ctypes.c_uint64(kmax),
             dptr(d_off) if D else None, dptr(dcl) if D else None, dptr(dk) if D else None)
    torch.cuda.current_stream(dev).synchronize()
    drow = torch.from_numpy(rows.astype(np.int32)).to(dev)
    return MapInput(clock, ec, vclk, vval, [0, D], drow, dcl, dk,
                    "contiguous block (crdt_device_alloc)" if block is not None else "torch caching allocator")


def orswot_op_streams(N: int, T: int, M: int, A: int, seed: int, p_rm: float = 0.2, p_future: float = 0.3,
                      rm_actors: int = 4, device="cuda"):
    """T ops per state for N states (an orswot.OrswotOpBatch, generated on `device` with torch's
    RNG): Op::Add of one member with the next dot of a random actor (the per-state count of
    that actor's adds so far, so every add is new), or w.p. p_rm an Op::Rm of one member whose
    clock keeps ~rm_actors actors of the state's clock at that point, with w.p. p_future one
    actor bumped past it (a remove from the future: deferred until that actor's next add)."""
    from .orswot import OrswotOpBatch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = N * T
    kind = (torch.rand((N, T), generator=g, device=device) < p_rm).to(torch.uint8)
    actor = torch.randint(0, A, (N, T), generator=g, device=device, dtype=torch.int64)
    onehot = torch.zeros((N, T, A), dtype=torch.int64, device=device)
    onehot.scatter_(2, actor.unsqueeze(2), (kind == 0).to(torch.int64).unsqueeze(2))
    cum = onehot.cumsum(1)  # adds of each actor up to and including op t
    del onehot
    counter = torch.gather(cum, 2, actor.unsqueeze(2)).squeeze(2)
    keep = torch.rand((N, T, A), generator=g, device=device) < (rm_actors / A)
    rm = torch.where(keep, cum, torch.zeros((), dtype=torch.int64, device=device))
    fut = (torch.rand((N, T), generator=g, device=device) < p_future).to(torch.int64)
    bump = torch.randint(0, A, (N, T, 1), generator=g, device=device)
    rm.scatter_add_(2, bump, fut.unsqueeze(2) * (1 + torch.gather(cum, 2, bump).squeeze(2) - torch.gather(
        rm, 2, bump).squeeze(2)).unsqueeze(2))
    del cum, keep
    member = torch.randint(0, M, (n,), generator=g, device=device, dtype=torch.int32)
    return OrswotOpBatch(
        op_off=torch.arange(N + 1, device=device, dtype=torch.int64) * T,
        kind=kind.reshape(n).contiguous(),
        actor=actor.reshape(n).to(torch.int32),
        counter=counter.reshape(n).contiguous(),
        rm_row=torch.arange(n, device=device, dtype=torch.int32),
        rm_clock=rm.reshape(n, A).contiguous(),
        mem_off=torch.arange(n + 1, device=device, dtype=torch.int64),
        mem=member)


def map_op_streams(N: int, T: int, K: int, A: int, seed: int, p_rm: float = 0.2, p_future: float = 0.3,
                   p_stale: float = 0.2, rm_actors: int = 4, device="cuda"):
    """T Map<K, MVReg> ops per state for N states (a map.MapOpBatch, generated on `device`):
    an Op::Up of a random key with the next dot of a random actor whose Put clock is the state's
    clock at that point plus the dot (a write with a fresh read ctx: it supersedes the key's
    values) or, w.p. p_stale, the clock of 1-8 ops earlier plus the dot (a write from a stale
    ctx: concurrent with what came since, so values accumulate); or w.p. p_rm an Op::Rm of one
    key with ~rm_actors actors of the state's clock, w.p. p_future from the future (deferred).
    Value = op index + 1."""
    from .map import MapOpBatch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = N * T
    i64 = torch.int64
    kind = (torch.rand((N, T), generator=g, device=device) < p_rm).to(torch.uint8)
    actor = torch.randint(0, A, (N, T), generator=g, device=device, dtype=i64)
    onehot = torch.zeros((N, T, A), dtype=i64, device=device)
    onehot.scatter_(2, actor.unsqueeze(2), (kind == 0).to(i64).unsqueeze(2))
    cum = onehot.cumsum(1)  # the state's clock after op t (ops applied in order)
    del onehot
    counter = torch.gather(cum, 2, actor.unsqueeze(2)).squeeze(2)
    stale = torch.rand((N, T), generator=g, device=device) < p_stale
    lag = torch.randint(1, 9, (N, T), generator=g, device=device) * stale
    src = (torch.arange(T, device=device).unsqueeze(0) - lag).clamp(min=0)
    put = torch.gather(cum, 1, src.unsqueeze(2).expand(N, T, A)).clone()
    put.scatter_(2, actor.unsqueeze(2), counter.unsqueeze(2))  # the Put's clock holds its own dot
    keep = torch.rand((N, T, A), generator=g, device=device) < (rm_actors / A)
    rm = torch.where(keep, cum, torch.zeros((), dtype=i64, device=device))
    fut = (torch.rand((N, T), generator=g, device=device) < p_future).to(i64)
    bump = torch.randint(0, A, (N, T, 1), generator=g, device=device)
    rm.scatter_(2, bump, torch.gather(rm, 2, bump) + fut.unsqueeze(2) * (
        1 + torch.gather(cum, 2, bump) - torch.gather(rm, 2, bump)))
    pool = torch.where((kind == 0).unsqueeze(2), put, rm).reshape(n, A).contiguous()
    del cum, keep, put, rm
    key = torch.randint(0, K, (n,), generator=g, device=device, dtype=torch.int32)
    return MapOpBatch(op_off=torch.arange(N + 1, device=device, dtype=i64) * T, kind=kind.reshape(n).contiguous(),
                      actor=actor.reshape(n).to(torch.int32), counter=counter.reshape(n).contiguous(), key=key,
                      val=torch.arange(1, n + 1, device=device, dtype=i64),
                      clk_row=torch.arange(n, device=device, dtype=torch.int32), clk_pool=pool,
                      key_off=torch.arange(n + 1, device=device, dtype=i64), keys=key)
