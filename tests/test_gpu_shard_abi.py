"""GPU: the C ABI's own RCCL sharded lub (crdt_*_lub_many_sharded, crdt_orswot_lub_many_sharded)
at world size 1 on one MI355X — the communicator setup, the exchange calls and the re-merge
bookkeeping (deferred pooling by group, survivor compaction) run for real; the multi-rank data
movement is the torch.distributed twin's, which tests/test_dist_cpu.py covers under gloo."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host, umax_torch

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


@pytest.fixture(scope="module")
def comm_ctx():
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    cg.shard.comm_init(ctx, cg.shard.unique_id(), 1, 0)
    assert cg.shard.comm_info(ctx) == (1, 0)
    yield ctx
    cg.shard.comm_destroy(ctx)
    assert cg.shard.comm_info(ctx) == (0, -1)
    ctx.close()


def test_sharded_needs_comm(gpu_ctx):
    x = torch.zeros((4, 8), dtype=torch.int64, device="cuda:0")
    with pytest.raises(cg.CrdtGpuError):
        cg.shard.lub_many_sharded("vclock", x, ctx=cg.Context(0))


@pytest.mark.parametrize("kind,W", [("vclock", 64), ("gcounter", 256), ("pncounter", 2 * 33), ("gset", 17)])
@pytest.mark.parametrize("G,R", [(1, 1000), (3, 77), (2, 0)])
def test_lattice_sharded_world1(comm_ctx, kind, W, G, R):
    rows = O.synth_matrix(0x5EED0011 + W, G * R, W, 1 if kind == "gset" else 0).reshape(G, R, W)
    x = to_dev(rows)
    got = to_host(cg.shard.lub_many_sharded(kind, x, ctx=comm_ctx))
    if R == 0:
        exp = np.zeros((G, W), np.uint64)
    elif kind == "gset":
        exp = np.bitwise_or.reduce(rows, axis=1)
    else:
        exp = to_host(umax_torch(x, 1))
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("seed,G,R,M,A", [(1, 1, 40, 64, 8), (2, 3, 12, 50, 8), (3, 2, 1, 130, 65)])
def test_orswot_sharded_world1(comm_ctx, seed, G, R, M, A):
    parts = [O.gen_orswot(seed * 10 + g, R, M, A, kmax=10, p_def=0.4) for g in range(G)]
    clock = np.stack([p[0] for p in parts])
    entries = np.stack([p[1] for p in parts])
    off = [0]
    for p in parts:
        off.append(off[-1] + p[3].shape[0])
    Mw = (M + 63) // 64
    dcl = np.concatenate([p[3] for p in parts]).reshape(-1, A)
    dmem = np.concatenate([p[4] for p in parts]).reshape(-1, Mw)
    kw = dict(def_off=off, def_clock=to_dev(dcl), def_members=to_dev(dmem)) if off[-1] else {}
    res = cg.shard.orswot_lub_many_sharded(to_dev(clock), to_dev(entries), ctx=comm_ctx, **kw)
    got_c, got_e = to_host(res.clock), to_host(res.entries)
    got_d = cg.shard.deferred_groups(res, G)
    for g, (c, e, o, d, m) in enumerate(parts):
        oc, oe, odef, _ = O.orswot_fold(c, e, o, d, m)
        np.testing.assert_array_equal(got_c[g], oc)
        np.testing.assert_array_equal(got_e[g], oe)
        assert got_d[g] == odef, g
    # a too-small def_cap is retried with exactly enough room
    small = cg.shard.orswot_lub_many_sharded(to_dev(clock), to_dev(entries), ctx=comm_ctx, def_cap=1, **kw)
    assert cg.shard.deferred_groups(small, G) == got_d
