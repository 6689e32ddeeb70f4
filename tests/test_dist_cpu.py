"""World-size-2 gloo tests of the replica-sharded exchange (crdts_gpu.dist) on CPU.

The local fold is injected with the oracle (the checker) because this host has no GPU; what
is under test is the sharding and the exchange step: sign-biased MAX all-reduce for the
counter lattices, all-gather + re-merge for GSet."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_local(kind):
    import oracle as O

    def f(shard):
        a = shard.numpy().view(np.uint64)
        if a.ndim == 2:
            out = O.gset_fold(a)[0] if kind == "gset" else O.vclock_fold(a)[0]
        else:
            out = np.stack([O.gset_fold(x)[0] if kind == "gset" else O.vclock_fold(x)[0] for x in a])
        return torch.from_numpy(out.view(np.int64).copy())
    return f


def _worker(rank, world, port, kind, R, W, G, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(here, ".."), os.path.join(here, "..", "rust-crdt_amd"), os.path.join(here, "..", "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from crdts_gpu import dist as cdist
    full = O.synth_matrix(0x5EED0005, G * R, W, 1 if kind == "gset" else 0).reshape(G, R, W)
    lo, hi = cdist.shard_range(R, rank, world)
    shard = torch.from_numpy(full[:, lo:hi].view(np.int64).copy())
    if G == 1:
        shard = shard[0]
    out = cdist.lub_many_sharded(kind, shard, local_lub=_oracle_local(kind))
    if rank == 0:
        q.put(out.numpy().view(np.uint64).copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,R,W,G", [("gcounter", 101, 16, 1), ("vclock", 64, 9, 3),
                                         ("pncounter", 50, 24, 1), ("gset", 77, 5, 1), ("gset", 20, 3, 2)])
def test_sharded_lub_world2(kind, R, W, G):
    import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, R, W, G, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = O.synth_matrix(0x5EED0005, G * R, W, 1 if kind == "gset" else 0).reshape(G, R, W)
    fold = O.gset_fold if kind == "gset" else O.vclock_fold
    exp = np.stack([fold(full[g])[0] for g in range(G)])
    np.testing.assert_array_equal(got.reshape(G, W), exp)


def test_shard_range_partitions():
    from crdts_gpu.dist import shard_range
    for R in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(R, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == R
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


def test_sign_bias_preserves_unsigned_order():
    from crdts_gpu.dist import _bias
    vals = np.array([0, 1, 2**63 - 1, 2**63, 2**64 - 1, 12345], dtype=np.uint64)
    t = torch.from_numpy(vals.view(np.int64).copy())
    b = _bias(t)
    order_u = np.argsort(vals, kind="stable")
    order_s = np.argsort(b.numpy(), kind="stable")
    assert (order_u == order_s).all()
