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


def allreduce_umax_(partial: torch.Tensor, group=None) -> torch.Tensor:
    """In-place unsigned-64 max all-reduce of an int64 tensor holding u64 bits."""
    if partial.dtype != torch.int64:
        raise TypeError("allreduce_umax_: int64 tensor holding u64 bits expected")
    b = _bias(partial)
    dist.all_reduce(b, op=dist.ReduceOp.MAX, group=group)
    partial.copy_(_bias(b))
    return partial


def allgather_rows(partial: torch.Tensor, group=None) -> torch.Tensor:
    """(…, W) partial -> (world, …, W) stacked in rank order."""
    world = dist.get_world_size(group)
    out = torch.empty((world,) + tuple(partial.shape), dtype=partial.dtype, device=partial.device)
    if dist.get_backend(group) == "gloo":  # gloo has no all_gather_into_tensor
        dist.all_gather(list(out.unbind(0)), partial.contiguous(), group=group)
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
