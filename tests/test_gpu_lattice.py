"""GPU parity: VClock / GCounter / PNCounter / GSet lub_many and merge_batch vs the oracle."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host, umax_torch

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402

SHAPES = [(1, 1), (2, 3), (3, 5), (17, 2), (1024, 64), (2048, 256), (5000, 256), (333, 1001),
          (700, 1024), (40, 1500), (4097, 6)]


@pytest.mark.parametrize("R,A", SHAPES)
def test_vclock_lub_many(gpu_ctx, R, A):
    rows = O.synth_matrix(0x5EED0001 + R, R, A, 0)
    exp, _ = O.vclock_fold(rows)
    got = to_host(cg.vclock.lub_many(to_dev(rows), ctx=gpu_ctx))
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("G,R,A", [(1, 9, 4), (7, 33, 20), (64, 5, 64), (300, 3, 7), (3, 3000, 256)])
def test_gcounter_lub_many_groups(gpu_ctx, G, R, A):
    x = O.synth_matrix(77 + G, G * R, A, 0).reshape(G, R, A)
    got = to_host(cg.gcounter.lub_many(to_dev(x), ctx=gpu_ctx))
    for g in range(G):
        exp, _ = O.vclock_fold(x[g])
        np.testing.assert_array_equal(got[g], exp)


def test_lub_strided_views_and_accumulate(gpu_ctx):
    big = O.synth_matrix(5, 300, 80, 0)
    dev = to_dev(big)
    view = dev[::3, 8:72]  # row stride 240 words, 64 columns, unaligned base (V=2 needs 16B)
    exp, _ = O.vclock_fold(big[::3, 8:72])
    np.testing.assert_array_equal(to_host(cg.vclock.lub_many(view, ctx=gpu_ctx)), exp)
    view2 = dev[::2, 1:64]  # odd base and odd width -> 8-byte path
    exp2, _ = O.vclock_fold(big[::2, 1:64])
    np.testing.assert_array_equal(to_host(cg.vclock.lub_many(view2, ctx=gpu_ctx)), exp2)
    # accumulate: out := out ⊔ fold(in)  ==  self.merge(r) for every r
    init = O.synth_matrix(6, 1, 64, 0)[0]
    out = to_dev(init.copy())
    cg.vclock.lub_many(view, out=out, accumulate=True, ctx=gpu_ctx)
    np.testing.assert_array_equal(to_host(out), np.maximum(init, exp))


def test_lub_empty(gpu_ctx):
    x = torch.empty((0, 16), dtype=torch.int64, device="cuda:0")
    out = cg.vclock.lub_many(x, ctx=gpu_ctx)
    assert to_host(out).tolist() == [0] * 16  # fold of nothing = VClock::new()
    x3 = torch.empty((4, 0, 8), dtype=torch.int64, device="cuda:0")
    out3 = torch.full((4, 8), 5, dtype=torch.int64, device="cuda:0")
    cg.vclock.lub_many(x3, out=out3, accumulate=True, ctx=gpu_ctx)
    assert (to_host(out3) == 5).all()


@pytest.mark.parametrize("R,A", [(1, 1), (100, 12), (4096, 256), (999, 33)])
def test_pncounter_lub_many(gpu_ctx, R, A):
    rows = O.synth_matrix(0x5EED0002 + A, R, 2 * A, 0)
    exp, _ = O.pncounter_fold(rows)
    got = to_host(cg.pncounter.lub_many(to_dev(rows), ctx=gpu_ctx))
    np.testing.assert_array_equal(got, exp)
    assert cg.pncounter.read(to_dev(got[None, :]))[0] == sum(int(v) for v in exp[:A]) - sum(int(v) for v in exp[A:])


@pytest.mark.parametrize("R,W", [(1, 1), (50, 3), (2000, 128), (123, 1025)])
def test_gset_lub_many(gpu_ctx, R, W):
    rows = O.synth_matrix(31 + W, R, W, 1)
    exp, _ = O.gset_fold(rows)
    got = to_host(cg.gset.lub_many(to_dev(rows), ctx=gpu_ctx))
    np.testing.assert_array_equal(got, exp)


# merge_batch launch forms: the flat 16-byte stream of packed rows (default, one workgroup per CU;
# mflat=4: four; mfu = 16-byte pieces per lane in flight: 2 by default, 1 or 4), and the row-group
# kernels (mflat=0, also the path of strided rows)
@pytest.mark.parametrize("mode", ["", "mflat=0", "mflat=4", "mfu=1", "mfu=4", "mflat=2,mfu=4"])
@pytest.mark.parametrize("N,A", [(1, 1), (10, 7), (7, 2), (33, 6), (1000, 64), (3000, 256), (64, 1030)])
def test_merge_batch(gpu_ctx, mode, N, A):
    if mode:
        gpu_ctx = cg.Context(0)
        gpu_ctx.tune(mode)
    s = O.synth_matrix(11, N, A, 0)
    o = O.synth_matrix(12, N, A, 0)
    exp = O.vclock_merge_pairs(s, o)
    ds = to_dev(s)
    cg.vclock.merge_batch(ds, to_dev(o), ctx=gpu_ctx)
    np.testing.assert_array_equal(to_host(ds), exp)
    gs = to_dev(O.synth_matrix(13, N, A, 1))
    go = O.synth_matrix(14, N, A, 1)
    exp_g = O.synth_matrix(13, N, A, 1) | go
    cg.gset.merge_batch(gs, to_dev(go), ctx=gpu_ctx)
    np.testing.assert_array_equal(to_host(gs), exp_g)
    ps = O.synth_matrix(15, N, 2 * A, 0)
    po = O.synth_matrix(16, N, 2 * A, 0)
    exp_p = O.vclock_merge_pairs(ps, po)
    dps = to_dev(ps)
    cg.pncounter.merge_batch(dps, to_dev(po), ctx=gpu_ctx)
    np.testing.assert_array_equal(to_host(dps), exp_p)
    # strided rows (views into wider buffers): never the flat stream
    wide = to_dev(np.concatenate([s, np.zeros((N, 2), np.uint64)], axis=1))
    owide = to_dev(np.concatenate([o, np.zeros((N, 2), np.uint64)], axis=1))
    cg.vclock.merge_batch(wide[:, :A], owide[:, :A], ctx=gpu_ctx)
    np.testing.assert_array_equal(to_host(wide[:, :A]), exp)
    assert not to_host(wide[:, A:]).any()


@pytest.mark.parametrize("rows,width,kind", [(3, 5, 0), (100, 256, 0), (7, 9, 1), (1, 1000, 2), (1, 1000, 3)])
def test_synth_fill_matches_cpu(gpu_ctx, rows, width, kind):
    t = torch.empty((rows, width), dtype=torch.int64, device="cuda:0")
    cg.synth_fill(gpu_ctx, t, 0x5EED0002, kind)
    np.testing.assert_array_equal(to_host(t), O.synth_matrix(0x5EED0002, rows, width, kind))


def test_config2_full_size_properties(gpu_ctx):
    """BASELINE config 2 at full size (1,048,576 x 256 u64 GCounter; PNCounter 2x256):
    sampled rows regenerated on the CPU, lub == torch unsigned max, lub is an upper bound of
    every sampled row, idempotent (accumulate with itself) and equal to the lub of two halves."""
    R, A = 1 << 20, 256
    x = torch.empty((R, A), dtype=torch.int64, device="cuda:0")
    cg.synth_fill(gpu_ctx, x, 0x5EED0002, 0)
    for r in (0, 1, 12345, R - 1):
        np.testing.assert_array_equal(to_host(x[r]), O.synth_matrix(0x5EED0002, 1, A, 0, row0=r)[0])
    out = cg.gcounter.lub_many(x, ctx=gpu_ctx)
    ref = umax_torch(x, 0)
    assert torch.equal(out, ref)
    h = to_host(out)
    sample = O.synth_matrix(0x5EED0002, 512, A, 0, row0=777)
    assert (sample <= h).all()
    again = out.clone()
    cg.gcounter.lub_many(x, out=again, accumulate=True, ctx=gpu_ctx)
    assert torch.equal(again, out)
    halves = torch.stack([cg.gcounter.lub_many(x[: R // 2], ctx=gpu_ctx),
                          cg.gcounter.lub_many(x[R // 2:], ctx=gpu_ctx)])
    assert torch.equal(cg.gcounter.lub_many(halves, ctx=gpu_ctx), out)
    del x
    y = torch.empty((R, 2 * A), dtype=torch.int64, device="cuda:0")
    cg.synth_fill(gpu_ctx, y, 0x5EED0003, 0)
    assert torch.equal(cg.pncounter.lub_many(y, ctx=gpu_ctx), umax_torch(y, 0))
