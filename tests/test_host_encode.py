"""CPU: the host-side op ingest (crdts_gpu.orswot.encode_ops / crdts_gpu.map.encode_ops) builds
the crdt_orswot_ops / crdt_map_ops CSR layout the kernels read (include/crdt_gpu.h)."""
import numpy as np

import crdts_gpu as cg


def test_orswot_encode_ops_layout():
    streams = [[("add", 2, 5, [1, 3]), ("rm", {0: 4, 2: 1}, [3])], [], [("rm", [0, 7, 0], [])]]
    b = cg.orswot.encode_ops(streams, 3, "cpu")
    assert b.op_off.tolist() == [0, 2, 2, 3]
    assert b.kind.tolist() == [0, 1, 1]
    assert b.actor.tolist()[0] == 2 and b.counter.tolist()[0] == 5
    assert b.mem_off.tolist() == [0, 2, 3, 3]
    assert b.mem.tolist()[:3] == [1, 3, 3]
    rc = b.rm_clock.numpy().view(np.uint64)
    assert rc[b.rm_row[1]].tolist() == [4, 0, 1] and rc[b.rm_row[2]].tolist() == [0, 7, 0]
    assert b.rm_clock.shape[0] >= 1 and b.mem.shape[0] >= 1  # never-empty device buffers


def test_map_encode_ops_layout():
    big = (1 << 64) - 1
    streams = [[("up", 1, 3, 4, {1: 3, 0: 2}, big), ("rm", {1: 9}, [4, 0])], [("up", 0, 1, 0, [1, 0], 7)]]
    b = cg.map.encode_ops(streams, 2, "cpu")
    assert b.op_off.tolist() == [0, 2, 3]
    assert b.kind.tolist() == [0, 1, 0]
    assert b.key.tolist() == [4, 0, 0] and b.actor.tolist() == [1, 0, 0]
    assert b.val.numpy().view(np.uint64).tolist() == [big, 0, 7]
    pool = b.clk_pool.numpy().view(np.uint64)
    assert [pool[r].tolist() for r in b.clk_row.tolist()] == [[2, 3], [0, 9], [1, 0]]
    assert b.key_off.tolist() == [0, 0, 2, 2] and b.keys.tolist()[:2] == [4, 0]


def test_synth_op_streams_shapes():
    o = cg.synth.orswot_op_streams(3, 8, 5, 4, seed=1, device="cpu")
    m = cg.synth.map_op_streams(3, 8, 5, 4, seed=1, device="cpu")
    for b in (o, m):
        assert b.op_off.tolist() == [0, 8, 16, 24] and b.kind.shape == (24,)
    # every add / up carries a fresh dot: counters of one actor rise by 1 within a state
    k, a, c = o.kind.view(3, 8), o.actor.view(3, 8), o.counter.view(3, 8)
    for s in range(3):
        seen = {}
        for t in range(8):
            if k[s, t] == 0:
                assert int(c[s, t]) == seen.get(int(a[s, t]), 0) + 1
                seen[int(a[s, t])] = int(c[s, t])
