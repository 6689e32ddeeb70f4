"""GPU: CmRDT::apply of Map<K, GCounter> / Map<K, PNCounter> (round 5; crdt_map_counter_apply_batch)
against the oracle's Map.apply (map.rs:119-137, apply_keyset_rm :318-348, apply_deferred :311-316,
gcounter.rs:36-42, pncounter.rs:59-68) on op-replay states with deferred removes: fresh, stale (seen)
and gapped dots, removes from the future (deferred, then re-applied by later Ups), equal rm clocks
(key sets unioned), malformed ops, and A past one lane word."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _streams(rng, maps, K, A, W, T):
    """Per-state op streams (the kernel's tuple form and the oracle's op objects)."""
    streams, oracle_ops = [], []
    for m in maps:
        clk = {a: m.clock.get(a) for a in range(A)}
        ops, oops, last_rm = [], [], None
        for _ in range(T):
            x = rng.random()
            if x < 0.7:  # Op::Up
                a = int(rng.integers(A))
                c = clk[a] + int(rng.integers(1, 3)) if rng.random() < 0.85 else max(clk[a] - int(rng.integers(0, 2)), 1)
                clk[a] = max(clk[a], c)
                k, va = int(rng.integers(K)), int(rng.integers(A))
                vc = int(rng.integers(1, 60))
                d = int(rng.integers(W))
                ops.append(("up", a, c, k, va, vc, d))
                vop = O.Dot(va, vc) if W == 1 else (O.Dot(va, vc), O.PNCounter.POS if d == 0 else O.PNCounter.NEG)
                oops.append(O.MapUp(O.Dot(a, c), k, vop))
            else:  # Op::Rm: a clock up to 2 ahead of ours on a few actors (deferred) or behind
                if last_rm is not None and rng.random() < 0.25:
                    row = last_rm  # an equal clock again: its key set is unioned
                else:
                    row = {a: max(0, clk[a] + int(rng.integers(-3, 3))) for a in range(A) if rng.random() < 0.5}
                    row = {a: c for a, c in row.items() if c}
                last_rm = row
                ks = sorted(set(int(z) for z in rng.choice(K, size=int(rng.integers(1, 4)), replace=False)))
                ops.append(("rm", row, ks))
                oops.append(O.MapRm(O.VClock(dict(row)), ks))
        streams.append(ops)
        oracle_ops.append(oops)
    return streams, oracle_ops


@pytest.mark.parametrize("W,A,seed", [(1, 6, 1), (2, 6, 2), (1, 70, 3), (2, 130, 4)])
def test_map_counter_apply(gpu_ctx, W, A, seed):
    N, K, T, Dcap = 24, 6, 40, 16
    maps = O.map_counter_objects(N, K, A, W, seed=40, steps=220) if A <= 6 else \
        O.map_counter_objects(N, K, A, W, seed=40 + seed, steps=260)
    d = O.map_counter_to_dense(maps, K, A, W)
    rng = np.random.default_rng(seed)
    streams, oracle_ops = _streams(rng, maps, K, A, W, T)
    Kw = (K + 63) // 64
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    for j in range(d["def_row"].shape[0]):  # the replicas' own deferred removes, as slots
        n = int(d["def_row"][j])
        dcl[n, cnt[n]] = d["def_clock"][j]
        dks[n, cnt[n]] = d["def_keys"][j]
        cnt[n] += 1
    clock, ec, val = to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["val"])
    tdc, tdk, tcnt = to_dev(dcl), to_dev(dks), torch.from_numpy(cnt).cuda()
    ops = cg.map.encode_counter_ops(streams, A, "cuda:0")
    status = cg.map.counter_apply_batch(clock, ec, val, tdc, tdk, tcnt, ops, ctx=gpu_ctx).cpu().numpy()
    c, e, v = to_host(clock), to_host(ec), to_host(val)
    hdc, hdk, hcnt = to_host(tdc), to_host(tdk), tcnt.cpu().numpy()
    deferred_seen = 0
    for n in range(N):
        exp = maps[n].copy()
        for op in oracle_ops[n]:
            exp.apply(op)
        assert status[n] == 0, (n, status[n])
        dfr = [(hdc[n, i], O.bitmap_members(hdk[n, i])) for i in range(int(hcnt[n]))]
        got = O.dense_to_map_counter(c[n], e[n], v[n], dfr)
        assert got == exp, n
        deferred_seen += len(exp.deferred)
    assert deferred_seen > 0


def test_map_counter_apply_malformed_and_capacity(gpu_ctx):
    """Malformed ops (actor / key / dir out of range, an rm row past the pool) are skipped and flagged
    (bit 1); a deferred list past Dcap is flagged (bit 0); a def_count past Dcap leaves the state
    untouched (bit 2)."""
    K, A, W = 4, 4, 2
    streams = [
        [("up", 9, 1, 0, 0, 1, 0), ("up", 0, 1, 9, 0, 1, 0), ("up", 0, 1, 0, 0, 1, 5), ("up", 1, 1, 2, 3, 7, 1)],
        [("rm", {0: 5 + i}, [i % K]) for i in range(3)],
        [("up", 0, 1, 0, 0, 1, 0)],
    ]
    ops = cg.map.encode_counter_ops(streams, A, "cuda:0")
    N, Dcap = 3, 2
    clock = torch.zeros((N, A), dtype=torch.int64, device="cuda:0")
    ec = torch.zeros((N, K, A), dtype=torch.int64, device="cuda:0")
    val = torch.zeros((N, K, W, A), dtype=torch.int64, device="cuda:0")
    dc = torch.zeros((N, Dcap, A), dtype=torch.int64, device="cuda:0")
    dk = torch.zeros((N, Dcap, 1), dtype=torch.int64, device="cuda:0")
    cnt = torch.tensor([0, 0, 3], dtype=torch.int32, device="cuda:0")
    st = cg.map.counter_apply_batch(clock, ec, val, dc, dk, cnt, ops, ctx=gpu_ctx).cpu().numpy()
    assert st[0] == 2 and st[1] == 1 and st[2] == 4
    v = to_host(val)
    assert v[0, 2, 1, 3] == 7 and to_host(ec)[0, 2, 1] == 1  # the one good op of state 0 applied
    assert int(cnt[1]) == 2 and to_host(clock)[2].sum() == 0


@pytest.mark.parametrize("W", [1, 2])
def test_map_counter_apply_unapplied_input_deferred(gpu_ctx, W):
    """Input states holding deferred removes never applied to their keys (the reference's apply_deferred
    still forgets those keys on the next Up): the kernel's first apply_deferred pass is a full one, the
    later ones re-forget the Up's own key only."""
    N, K, A, T, Dcap = 16, 5, 6, 12, 16
    maps = O.map_counter_objects(N, K, A, W, seed=40, steps=220)
    rng = np.random.default_rng(90 + W)
    for m in maps:  # a remove from the future naming present keys, not applied to them
        row = {a: m.clock.get(a) + 1 for a in range(2)}
        m.deferred[O.VClock(dict(row))] = set(int(k) for k in rng.choice(K, size=2, replace=False))
    d = O.map_counter_to_dense(maps, K, A, W)
    streams, oracle_ops = _streams(rng, maps, K, A, W, T)
    Kw = (K + 63) // 64
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    for j in range(d["def_row"].shape[0]):
        n = int(d["def_row"][j])
        dcl[n, cnt[n]], dks[n, cnt[n]] = d["def_clock"][j], d["def_keys"][j]
        cnt[n] += 1
    clock, ec, val = to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["val"])
    tdc, tdk, tcnt = to_dev(dcl), to_dev(dks), torch.from_numpy(cnt).cuda()
    ops = cg.map.encode_counter_ops(streams, A, "cuda:0")
    status = cg.map.counter_apply_batch(clock, ec, val, tdc, tdk, tcnt, ops, ctx=gpu_ctx).cpu().numpy()
    c, e, v = to_host(clock), to_host(ec), to_host(val)
    hdc, hdk, hcnt = to_host(tdc), to_host(tdk), tcnt.cpu().numpy()
    ups = 0
    for n in range(N):
        exp = maps[n].copy()
        for op in oracle_ops[n]:
            exp.apply(op)
        ups += sum(isinstance(op, O.MapUp) for op in oracle_ops[n])
        assert status[n] == 0, (n, status[n])
        dfr = [(hdc[n, i], O.bitmap_members(hdk[n, i])) for i in range(int(hcnt[n]))]
        assert O.dense_to_map_counter(c[n], e[n], v[n], dfr) == exp, n
    assert ups > 0


def test_map_counter_apply_offsets_past_the_key_pool(gpu_ctx):
    """A key_off whose last entry claims more keys than the pool holds: the bound is the
    pool's length, so the op is flagged (status bit 1) and skipped instead of read past the buffer;
    wrongly typed / short / host-resident op fields are refused on the host."""
    K, A, W, N, Dcap = 4, 4, 1, 2, 2
    streams = [[("rm", {0: 3}, [1])], [("up", 0, 1, 0, 0, 1, 0)]]
    ops = cg.map.encode_counter_ops(streams, A, "cuda:0")
    bad_off = ops.key_off.clone()
    bad_off[1:] = 1 << 20  # op 0 claims a million keys
    bad = ops._replace(key_off=bad_off)
    mk = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    clock, ec, val, dc, dk = mk(N, A), mk(N, K, A), mk(N, K, W, A), mk(N, Dcap, A), mk(N, Dcap, 1)
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda:0")
    st = cg.map.counter_apply_batch(clock, ec, val, dc, dk, cnt, bad, ctx=gpu_ctx).cpu().numpy()
    torch.cuda.synchronize()
    assert st[0] & 2 and st[1] == 0
    assert int(cnt[0]) == 0 and to_host(ec)[1, 0, 0] == 1
    with pytest.raises(TypeError):
        cg.map.counter_apply_batch(clock, ec, val, dc, dk, cnt, ops._replace(counter=ops.counter.to(torch.int32)),
                                   ctx=gpu_ctx)
    with pytest.raises(ValueError):
        cg.map.counter_apply_batch(clock, ec, val, dc, dk, cnt, ops._replace(key=ops.key[:0]), ctx=gpu_ctx)
    with pytest.raises(ValueError):
        cg.map.counter_apply_batch(clock, ec, val, dc, dk, cnt, ops._replace(vdir=ops.vdir.cpu()), ctx=gpu_ctx)


def _future_rm_streams(rng, maps, K, A, W, T, p_rm=0.55):
    """Streams whose Rms carry clocks far ahead on actor 0 (distinct per op) while the Ups use actors
    1.. only: no Rm is ever dominated, so every one stays deferred (a long deferred list)."""
    streams, oracle_ops = [], []
    for m in maps:
        clk = {a: m.clock.get(a) for a in range(A)}
        ops, oops = [], []
        for i in range(T):
            if rng.random() < p_rm:
                row = {0: clk[0] + 1000 + i}
                if rng.random() < 0.5:
                    row[1] = max(1, clk[1])
                ks = sorted(set(int(z) for z in rng.choice(K, size=int(rng.integers(1, 4)), replace=False)))
                ops.append(("rm", row, ks))
                oops.append(O.MapRm(O.VClock(dict(row)), ks))
            else:
                a = int(rng.integers(1, A))
                c = clk[a] + int(rng.integers(1, 3))
                clk[a] = c
                k, va, vc, d = int(rng.integers(K)), int(rng.integers(A)), int(rng.integers(1, 60)), int(rng.integers(W))
                ops.append(("up", a, c, k, va, vc, d))
                vop = O.Dot(va, vc) if W == 1 else (O.Dot(va, vc), O.PNCounter.POS if d == 0 else O.PNCounter.NEG)
                oops.append(O.MapUp(O.Dot(a, c), k, vop))
        streams.append(ops)
        oracle_ops.append(oops)
    return streams, oracle_ops


@pytest.mark.parametrize("W", [1, 2])
def test_map_counter_apply_long_deferred_list(gpu_ctx, W):
    """More deferred removes than the 16 slots the kernel holds in LDS (round 6: slots 16 .. Dcap-1 are
    used in place in the caller's slot arrays): with Dcap = 48 every state ends with 20+ removes and
    status 0, equal to the oracle's Map.apply; Dcap = 16 on the same streams flags bit 0."""
    N, K, A, T = 10, 6, 5, 64
    maps = O.map_counter_objects(N, K, A, W, seed=44, steps=120)
    d = O.map_counter_to_dense(maps, K, A, W)
    rng = np.random.default_rng(7 + W)
    streams, oracle_ops = _future_rm_streams(rng, maps, K, A, W, T)
    Kw = (K + 63) // 64
    for Dcap in (48, 16):
        dcl = np.zeros((N, Dcap, A), np.uint64)
        dks = np.zeros((N, Dcap, Kw), np.uint64)
        cnt = np.zeros(N, np.int32)
        for j in range(d["def_row"].shape[0]):
            n = int(d["def_row"][j])
            dcl[n, cnt[n]] = d["def_clock"][j]
            dks[n, cnt[n]] = d["def_keys"][j]
            cnt[n] += 1
        clock, ec, val = to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["val"])
        tdc, tdk, tcnt = to_dev(dcl), to_dev(dks), torch.from_numpy(cnt).cuda()
        ops = cg.map.encode_counter_ops(streams, A, "cuda:0")
        status = cg.map.counter_apply_batch(clock, ec, val, tdc, tdk, tcnt, ops, ctx=gpu_ctx).cpu().numpy()
        if Dcap == 16:
            assert (status & 1).all()  # every state ran past 16 removes
            continue
        c, e, v = to_host(clock), to_host(ec), to_host(val)
        hdc, hdk, hcnt = to_host(tdc), to_host(tdk), tcnt.cpu().numpy()
        longest = 0
        for n in range(N):
            exp = maps[n].copy()
            for op in oracle_ops[n]:
                exp.apply(op)
            assert status[n] == 0, (n, status[n])
            dfr = [(hdc[n, i], O.bitmap_members(hdk[n, i])) for i in range(int(hcnt[n]))]
            assert O.dense_to_map_counter(c[n], e[n], v[n], dfr) == exp, n
            longest = max(longest, len(exp.deferred))
        assert 20 <= longest <= 48


def test_map_counter_apply_vacated_slots_zeroed(gpu_ctx):
    """A deferred list that grows past the 16 LDS slots and then empties (a last Up on actor 0 from
    and actor 1 from past every remove's clock dominate them all): count 0, every slot written back zero (the form
    the wire ingest produces), state equal to the oracle's Map.apply."""
    N, K, A, T, W, Dcap = 6, 6, 5, 64, 2, 48
    maps = O.map_counter_objects(N, K, A, W, seed=45, steps=0)
    d = O.map_counter_to_dense(maps, K, A, W)
    rng = np.random.default_rng(9)
    streams, oracle_ops = _future_rm_streams(rng, maps, K, A, W, T)
    for s, oo in zip(streams, oracle_ops):
        for a in (1, 0):  # (the removes' clocks name actors 0 and 1 only)
            s.append(("up", a, 1 << 20, 0, 1, 1, 0))
            oo.append(O.MapUp(O.Dot(a, 1 << 20), 0, (O.Dot(1, 1), O.PNCounter.POS)))
    Kw = (K + 63) // 64
    clock, ec, val = to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["val"])
    tdc, tdk = to_dev(np.zeros((N, Dcap, A), np.uint64)), to_dev(np.zeros((N, Dcap, Kw), np.uint64))
    tcnt = torch.zeros(N, dtype=torch.int32, device="cuda:0")
    ops = cg.map.encode_counter_ops(streams, A, "cuda:0")
    status = cg.map.counter_apply_batch(clock, ec, val, tdc, tdk, tcnt, ops, ctx=gpu_ctx).cpu().numpy()
    assert (status == 0).all(), status
    assert (tcnt.cpu().numpy() == 0).all()
    assert not to_host(tdc).any() and not to_host(tdk).any()
    c, e, v = to_host(clock), to_host(ec), to_host(val)
    for n in range(N):
        exp = maps[n].copy()
        for op in oracle_ops[n]:
            exp.apply(op)
        assert not exp.deferred
        assert O.dense_to_map_counter(c[n], e[n], v[n], []) == exp, n
