"""GPU parity of the multi-segment lattice lub (crdt_lub_many_multi): several VClock / GCounter /
PNCounter / GSet folds in one launch per join op must write exactly what one
crdt_<kind>_lub_many call per segment writes (vclock.rs:130-136, pncounter.rs:70-75,
gset.rs:38-40): mixed kinds and vector widths, strided views, groups, empty folds, accumulate, more
segments than one launch holds, and the sharded form at world size 1."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def fold(kind, rows):
    """Oracle fold of (R, W) host rows (or (G, R, W))."""
    if rows.ndim == 3:
        return np.stack([fold(kind, r) for r in rows]) if rows.shape[0] else np.zeros((0, rows.shape[2]), np.uint64)
    if rows.shape[0] == 0:
        return np.zeros(rows.shape[1], np.uint64)
    if kind == "gset":
        return O.gset_fold(rows)[0]
    if kind == "pncounter":
        return O.pncounter_fold(rows)[0]
    return O.vclock_fold(rows)[0]


CASES = [("gcounter", 1, 2000, 256), ("pncounter", 1, 700, 2 * 100), ("vclock", 3, 77, 63), ("gset", 2, 300, 5),
         ("vclock", 1, 0, 8), ("gcounter", 40, 9, 130), ("vclock", 1, 1, 2), ("gset", 1, 4097, 64),
         ("pncounter", 5, 33, 2 * 7), ("vclock", 2, 1000, 1024), ("gcounter", 1, 65536, 6)]


def make(i, kind, G, R, W):
    rows = O.synth_matrix(0x5EED0061 + i, G * R, W, 1 if kind == "gset" else 0).reshape(G, R, W)
    return rows


def test_multi_matches_per_type(gpu_ctx):
    items, exps = [], []
    for i, (kind, G, R, W) in enumerate(CASES):
        rows = make(i, kind, G, R, W)
        x = to_dev(rows if G > 1 else rows[0])
        out = torch.full((G, W) if G > 1 else (W,), 7, dtype=torch.int64, device="cuda")
        items.append((kind, x, out))
        exps.append(fold(kind, rows if G > 1 else rows[0]))
    cg.lub_many_multi(items, ctx=gpu_ctx)
    for (kind, _, out), exp in zip(items, exps):
        np.testing.assert_array_equal(to_host(out), exp, err_msg=kind)


def test_multi_strided_and_accumulate(gpu_ctx):
    big = O.synth_matrix(0x5EED0071, 600, 80, 0)
    dev = to_dev(big)
    views = [("vclock", dev[::3, 8:72]), ("gcounter", dev[1::2, 1:64]), ("pncounter", dev[:500, :80])]
    start = [O.synth_matrix(0x5EED0072 + i, 1, v.shape[1], 0)[0] for i, (_, v) in enumerate(views)]
    items = [(k, v, to_dev(s0)) for (k, v), s0 in zip(views, start)]
    cg.lub_many_multi(items, ctx=gpu_ctx, accumulate=True)
    for (kind, v, out), s0 in zip(items, start):
        exp = fold(kind, np.concatenate([s0[None], to_host(v)]))
        np.testing.assert_array_equal(to_host(out), exp, err_msg=kind)


def test_multi_more_segments_than_one_launch(gpu_ctx):
    items, exps = [], []
    for i in range(19):  # 19 max segments: three launches of <= 8
        rows = make(100 + i, "gcounter", 1, 50 + 37 * i, 24)
        items.append(("gcounter", to_dev(rows[0]), torch.empty(24, dtype=torch.int64, device="cuda")))
        exps.append(fold("gcounter", rows[0]))
    gpu_ctx.set_timing(True)
    gpu_ctx.timing_reset()
    cg.lub_many_multi(items, ctx=gpu_ctx)
    ms, n = gpu_ctx.timing("lub_stream")
    gpu_ctx.set_timing(False)
    assert n == 3
    for (_, _, out), exp in zip(items, exps):
        np.testing.assert_array_equal(to_host(out), exp)


def test_multi_bench_shape(gpu_ctx):
    """bench.py's step: GCounter 1M x 256 + PNCounter 1M x 2x256 in one launch."""
    R, A = 1 << 20, 256
    g = torch.empty((R, A), dtype=torch.int64, device="cuda")
    p = torch.empty((R, 2 * A), dtype=torch.int64, device="cuda")
    cg.synth_fill(gpu_ctx, g, 0x5EED0002, 0)
    cg.synth_fill(gpu_ctx, p, 0x5EED0003, 0)
    og, op = (torch.empty(w, dtype=torch.int64, device="cuda") for w in (A, 2 * A))
    cg.lub_many_multi([("gcounter", g, og), ("pncounter", p, op)], ctx=gpu_ctx)
    np.testing.assert_array_equal(to_host(og), to_host(cg.gcounter.lub_many(g, ctx=gpu_ctx)))
    np.testing.assert_array_equal(to_host(op), to_host(cg.pncounter.lub_many(p, ctx=gpu_ctx)))


def test_multi_sharded_world1():
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    cg.shard.comm_init(ctx, cg.shard.unique_id(), 1, 0)
    try:
        items, exps = [], []
        for i, (kind, G, R, W) in enumerate([("gcounter", 1, 3000, 256), ("pncounter", 2, 100, 66), ("gset", 3, 50, 9)]):
            rows = make(200 + i, kind, G, R, W)
            items.append((kind, to_dev(rows if G > 1 else rows[0]),
                          torch.empty((G, W) if G > 1 else (W,), dtype=torch.int64, device="cuda")))
            exps.append(fold(kind, rows if G > 1 else rows[0]))
        cg.shard.lub_many_multi_sharded(items, ctx=ctx)
        for (kind, _, out), exp in zip(items, exps):
            np.testing.assert_array_equal(to_host(out), exp, err_msg=kind)
    finally:
        cg.shard.comm_destroy(ctx)
        ctx.close()


def test_multi_rejects_bad_kind(gpu_ctx):
    from crdts_gpu import _abi
    arr = (_abi.LubSegment * 1)()
    arr[0].kind = 99
    with pytest.raises(cg.CrdtGpuError):
        gpu_ctx.call("crdt_lub_many_multi", arr, 1)
