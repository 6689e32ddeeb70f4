"""GPU parity: batched Map<K, MVReg<u64>> CmRDT::apply (crdt_map_apply_batch) vs the oracle's
one-by-one Map.apply (map.rs:119-137, apply_keyset_rm :318-348, MVReg::apply mvreg.rs:130-166).

Op streams come from op replay with the reference's ctx API (writes with the ctx of get(key),
removes with an rm ctx read here or at another replica, test/map.rs:71-146 style), delivered to
each state as a random subset in perturbed causal order and cut at a random point, so removes
defer and concurrent writes leave several values per register."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


@pytest.fixture(scope="module", params=["alane=1", "alane=1,mameta=0", "alane=1,mapf=0", "alane=0"])
def mactx(request):
    """Both kernels: 16 lanes per state (alane=1, the default for A <= 64; mapf=0 without the
    next op's entry-row prefetch) and one wave per state (alane=0, every A); shapes with A > 64
    take the wave kernel in every mode."""
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    ctx.tune(request.param)
    yield ctx
    ctx.close()






def replay_streams(seed, n_states, n_origins, K, n_ops, rm_heavy=False, key_stride=1):
    """rm_heavy: keep most removes and few writes, in causal order, so removes whose context saw
    dropped writes pile up in the deferred list."""
    rng = np.random.default_rng(seed)
    origins = [O.Map(O.MVReg) for _ in range(n_origins)]
    ops, val = [], 1
    for _ in range(n_ops):
        a = int(rng.integers(n_origins))
        m = origins[a]
        x = rng.random()
        if x < 0.1:
            m.merge(origins[int(rng.integers(n_origins))])
            continue
        k = int(rng.integers(K // key_stride)) * key_stride
        if x < 0.75:
            op = m.update(k, m.get(k).derive_add_ctx(a), lambda r, c, v=val: r.write(v, c))
            val += 1
        else:
            src = m if rng.random() < 0.5 else origins[int(rng.integers(n_origins))]
            op = m.rm(k, src.get(k).derive_rm_ctx())
        m.apply(op)
        ops.append(op)
    streams = []
    if rm_heavy:
        for _ in range(n_states):
            p_up = rng.uniform(0.1, 0.4)
            streams.append([op for op in ops if rng.random() < (p_up if isinstance(op, O.MapUp) else 0.95)])
        return streams
    for _ in range(n_states):
        keep = np.flatnonzero(rng.random(len(ops)) < rng.uniform(0.4, 1.0))
        idx = keep[np.argsort(keep + rng.normal(0, rng.uniform(0, 10), size=keep.shape[0]))]
        idx = idx[:int(rng.integers(len(idx) // 2, len(idx) + 1))]
        streams.append([ops[i] for i in idx])
    return streams


def op_tuple(op):
    if isinstance(op, O.MapUp):
        return ("up", op.dot.actor, op.dot.counter, op.key, dict(op.op.clock.dots), op.op.val)
    return ("rm", dict(op.clock.dots), sorted(op.keyset))


def oracle_apply(streams):
    out, peak = [], 1
    for ops in streams:
        m = O.Map(O.MVReg)
        for op in ops:
            m.apply(op)
            peak = max([peak] + [len(e.val.vals) for e in m.entries.values()])
        out.append(m)
    return out, peak


def gpu_apply(ctx, streams, K, A, V, Dcap):
    N = len(streams)
    Kw = (K + 63) // 64
    z = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    clock, ec, vclk, vval = z(N, A), z(N, K, A), z(N, K, V, A), z(N, K, V)
    dcl, dks = z(N, Dcap, A), z(N, Dcap, Kw)
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda:0")
    ops = cg.map.encode_ops([[op_tuple(o) for o in s] for s in streams], A, "cuda:0")
    status = cg.map.apply_batch(clock, ec, vclk, vval, dcl, dks, cnt, ops, ctx=ctx)
    torch.cuda.synchronize()
    c, e, vc, vv = to_host(clock), to_host(ec), to_host(vclk), to_host(vval)
    dc, dk, n = to_host(dcl), to_host(dks), cnt.cpu().numpy()
    maps = []
    for s in range(N):
        deferred = [(dc[s, d], O.bitmap_members(dk[s, d])) for d in range(int(n[s]))]
        maps.append((O.dense_to_map(c[s], e[s], vc[s], vv[s], deferred), vc[s], vv[s], e[s]))
    return maps, status.cpu().numpy()


@pytest.mark.parametrize("seed,n_states,n_origins,K,n_ops", [
    (1, 48, 3, 6, 80), (2, 100, 5, 20, 150), (3, 16, 70, 40, 300), (4, 64, 2, 2, 120)])
def test_map_apply_replay(mactx, seed, n_states, n_origins, K, n_ops):
    streams = replay_streams(seed, n_states, n_origins, K, n_ops)
    exp, peak = oracle_apply(streams)
    Dcap = max(1, max(sum(1 for o in s if isinstance(o, O.MapRm)) for s in streams))
    got, status = gpu_apply(mactx, streams, K, n_origins, min(peak, 8), min(Dcap, 24))
    assert (status == 0).all(), status
    assert sum(len(m.deferred) for m in exp) > 0 or seed in (1, 4)
    for s, ((g, vc, vv, ec), e) in enumerate(zip(got, exp)):
        assert g.clock == e.clock and g.entries == e.entries, s
        assert g.deferred == e.deferred, s
        # the value slots keep Vec order: the kernel's used slots in index order == oracle's vals
        for k, ent in e.entries.items():
            used = [j for j in range(vc.shape[1]) if vc[k, j].any()]
            assert [int(vv[k, j]) for j in used] == [v for _, v in ent.val.vals], (s, k)
        assert not vc[~ec.any(axis=1)].any()


@pytest.mark.parametrize("seed", [5, 6])
def test_map_apply_same_key_runs(mactx, seed):
    """Arbitrary ops (not ctx-derived) on 3 keys: runs of Ups and multi-key Rms on the same key
    back to back, so the prefetched entry row of the next op is often stale (written by the op
    before it) and must be reloaded; Rm keysets of 1-3 keys with the first key prefetched."""
    rng = np.random.default_rng(seed)
    A, K, N, T = 20, 3, 64, 48
    streams = []
    for _ in range(N):
        ops, ctr = [], {}
        for _ in range(T):
            clk = O.VClock({int(a): int(rng.integers(1, 6)) for a in rng.choice(A, size=int(rng.integers(0, 4)),
                                                                                   replace=False)})
            if rng.random() < 0.6:
                a = int(rng.integers(A))
                ctr[a] = ctr.get(a, 0) + int(rng.integers(1, 3))
                ops.append(O.MapUp(O.Dot(a, ctr[a]), int(rng.integers(K)), O.MVRegPut(clk, int(rng.integers(1, 1 << 40)))))
            else:
                ks = set(int(k) for k in rng.choice(K, size=int(rng.integers(1, 4)), replace=False))
                ops.append(O.MapRm(clk, ks))
        streams.append(ops)
    exp, peak = oracle_apply(streams)
    got, status = gpu_apply(mactx, streams, K, A, min(peak, 16), 48)
    assert (status == 0).all(), status
    for s, ((g, vc, vv, ec), e) in enumerate(zip(got, exp)):
        assert g.clock == e.clock and g.entries == e.entries, s
        assert g.deferred == e.deferred, s
        assert not vc[~ec.any(axis=1)].any()


def test_map_apply_value_overflow(mactx):
    # two concurrent writes to one key need 2 value slots
    a, b = O.Map(O.MVReg), O.Map(O.MVReg)
    op1 = a.update(0, a.get(0).derive_add_ctx(0), lambda r, c: r.write(11, c))
    op2 = b.update(0, b.get(0).derive_add_ctx(1), lambda r, c: r.write(22, c))
    got, status = gpu_apply(mactx, [[op1, op2], [op1]], 1, 2, 1, 1)
    assert status[0] & 16 and status[1] == 0
    exp, _ = oracle_apply([[op1, op2], [op1]])
    assert got[1][0].entries == exp[1].entries
    got, status = gpu_apply(mactx, [[op1, op2]], 1, 2, 2, 1)
    assert status[0] == 0 and got[0][0].entries == oracle_apply([[op1, op2]])[0][0].entries


def test_map_apply_key_range_past_buffer(mactx):
    """An Rm whose key range runs past the n_keys entries of `keys` (or is reversed) is malformed
    (status bit 1) and skipped without reading past the buffer; the rest of the stream applies."""
    a = O.Map(O.MVReg)
    up = a.update(1, a.get(1).derive_add_ctx(0), lambda r, c: r.write(7, c))
    a.apply(up)
    rm = a.rm(1, a.get(1).derive_rm_ctx())
    up2 = a.update(2, a.get(2).derive_add_ctx(0), lambda r, c: r.write(8, c))
    streams = [[up, rm, up2], [up, rm]]
    K, A, V, Dcap = 4, 2, 2, 2
    N, Kw = len(streams), 1
    z = lambda *s: torch.zeros(s, dtype=torch.int64, device="cuda:0")  # noqa: E731
    clock, ec, vclk, vval, dcl, dks = z(N, A), z(N, K, A), z(N, K, V, A), z(N, K, V), z(N, Dcap, A), z(N, Dcap, Kw)
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda:0")
    ops = cg.map.encode_ops([[op_tuple(o) for o in s] for s in streams], A, "cuda:0")
    n_keys = ops.keys.shape[0]
    ops.key_off[2] = n_keys + 4096     # state 0's Rm (op 1): range far past keys
    ops.key_off[5] = n_keys + 1        # state 1's Rm (op 4, the last op): one past the end
    status = cg.map.apply_batch(clock, ec, vclk, vval, dcl, dks, cnt, ops, ctx=mactx).cpu().numpy()
    torch.cuda.synchronize()
    assert status.tolist() == [2, 2]
    exp, _ = oracle_apply([[up, up2], [up]])
    c, e, vc, vv = to_host(clock), to_host(ec), to_host(vclk), to_host(vval)
    for s in range(N):
        assert int(cnt[s]) == 0
        assert O.dense_to_map(c[s], e[s], vc[s], vv[s], []) == exp[s], s


# A = 8 / 16 / 17 / 32 / 33 run the one-word-per-lane kernel, 100 the two-word one, 200 the four-word one
@pytest.mark.parametrize("N,T,K,A,V", [(256, 64, 16, 8, 4), (64, 100, 70, 33, 6), (48, 80, 24, 100, 8),
                                       (32, 80, 20, 200, 8), (257, 64, 16, 32, 4), (130, 70, 30, 16, 4),
                                       (99, 64, 20, 17, 4)])
def test_map_apply_synth_streams(mactx, N, T, K, A, V):
    """The bench's device-generated streams (crdts_gpu.synth.map_op_streams) vs the oracle."""
    b = cg.synth.map_op_streams(N, T, K, A, seed=N + K, device="cuda:0")
    h = {f: getattr(b, f).cpu().numpy() for f in b._fields}
    streams = []
    for s in range(N):
        ops = []
        for o in range(int(h["op_off"][s]), int(h["op_off"][s + 1])):
            row = h["clk_pool"][h["clk_row"][o]].view(np.uint64)
            clk = O.VClock({a: int(v) for a, v in enumerate(row) if v})
            k = int(h["keys"][h["key_off"][o]])
            ops.append(O.MapUp(O.Dot(int(h["actor"][o]), int(h["counter"][o])), k, O.MVRegPut(clk, int(h["val"][o])))
                       if h["kind"][o] == 0 else O.MapRm(clk, {k}))
        streams.append(ops)
    exp, peak = oracle_apply(streams)
    assert peak <= V
    got, status = gpu_apply(mactx, streams, K, A, V, 16)
    assert (status == 0).all()
    assert sum(len(m.deferred) for m in exp) > 0
    for s, ((g, _, _, _), e) in enumerate(zip(got, exp)):
        assert g == e, s


@pytest.mark.parametrize("hot", [0, 1, 3])
def test_map_apply_deferred_spill(hot):
    """Deferred slots beyond the LDS-resident ones live in the state's own HBM slots (CRDT_TUNE
    mhot=N): the same results with none, one or three slots in LDS."""
    ctx = cg.Context(0)
    ctx.tune(f"mhot={hot},alane=0")  # (LDS-resident slots: the wave-per-state kernel)
    try:
        streams = replay_streams(20 + hot, 40, 5, 20, 200, rm_heavy=True)
        exp, peak = oracle_apply(streams)
        Dcap = max(1, max(sum(1 for o in s if isinstance(o, O.MapRm)) for s in streams))
        assert max(len(m.deferred) for m in exp) > max(hot, 1)
        got, status = gpu_apply(ctx, streams, 20, 5, min(peak, 8), min(Dcap, 24))
        assert (status == 0).all(), status
        for s, ((g, _, _, _), e) in enumerate(zip(got, exp)):
            assert g.clock == e.clock and g.entries == e.entries, s
            assert g.deferred == e.deferred, s
    finally:
        ctx.close()


def test_map_apply_wide_deferred_list():
    """A deferred list far wider than LDS (A = 70, K = 4,000: 133 words a slot; Dcap = 183 slots is
    190 KiB per state): the launch keeps the 61 slots that fit in 64 KiB in LDS and the rest in HBM
    instead of refusing (with mhot=0 nothing is in LDS: test_map_apply_deferred_spill)."""
    ctx = cg.Context(0)
    try:
        streams = replay_streams(35, 12, 70, 4000, 700, rm_heavy=True, key_stride=100)
        exp, peak = oracle_apply(streams)
        assert peak <= 8
        Dcap = max(sum(1 for o in s if isinstance(o, O.MapRm)) for s in streams)
        assert Dcap * (70 + 63) * 8 > 64 * 1024
        got, status = gpu_apply(ctx, streams, 4000, 70, 8, Dcap)
        assert (status == 0).all(), status
        for s, ((g, _, _, _), e) in enumerate(zip(got, exp)):
            assert g.clock == e.clock and g.entries == e.entries, s
            assert g.deferred == e.deferred, s
    finally:
        ctx.close()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_map_apply_unapplied_input_deferred(mactx, seed):
    """Input states whose deferred removes were never applied to their rows (the reference's own
    states always hold them applied): the first apply_deferred must re-forget every key of every
    slot, later ones only the updated key (map_apply.hip's restricted pass).  Long Up streams on
    random keys, some seen, some Rm ops in between."""
    rng = np.random.default_rng(seed)
    N, K, A, V, Dcap = 64, 8, 4, 4, 48
    Kw = 1
    clock = rng.integers(0, 6, size=(N, A)).astype(np.uint64)
    ec = np.zeros((N, K, A), np.uint64)
    vclk = np.zeros((N, K, V, A), np.uint64)
    vval = np.zeros((N, K, V), np.uint64)
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dks = np.zeros((N, Dcap, Kw), np.uint64)
    cnt = np.zeros(N, np.int32)
    states, streams = [], []
    for s in range(N):
        for k in range(K):
            if rng.random() < 0.6:
                row = np.minimum(rng.integers(0, 6, size=A).astype(np.uint64), clock[s])
                if row.any():
                    ec[s, k] = row
                    vclk[s, k, 0] = row
                    vval[s, k, 0] = rng.integers(1, 100)
        nd, seen = int(rng.integers(1, 4)), set()
        for _ in range(nd):
            rm = rng.integers(0, 9, size=A).astype(np.uint64)
            if not rm.any() or rm.tobytes() in seen:
                continue
            seen.add(rm.tobytes())
            keys = [k for k in range(K) if rng.random() < 0.5] or [0]
            dcl[s, cnt[s]] = rm
            dks[s, cnt[s], 0] = sum(1 << k for k in keys)
            cnt[s] += 1
        deferred = [(dcl[s, d], O.bitmap_members(dks[s, d])) for d in range(int(cnt[s]))]
        states.append(O.dense_to_map(clock[s], ec[s], vclk[s], vval[s], deferred))
        ops, cur = [], clock[s].copy()
        for _ in range(int(rng.integers(5, 40))):
            a, k = int(rng.integers(A)), int(rng.integers(K))
            if rng.random() < 0.15:
                rmc = rng.integers(0, 9, size=A).astype(np.uint64)
                rmc[int(rng.integers(A))] += 1  # a non-empty rm clock
                ops.append(O.MapRm(O.VClock({x: int(v) for x, v in enumerate(rmc) if v}), {k}))
                continue
            c = int(cur[a]) + 1 if rng.random() < 0.85 else max(1, int(cur[a]))
            cur[a] = max(cur[a], c)
            put = {x: int(v) for x, v in enumerate(np.minimum(cur, rng.integers(0, 9, size=A))) if v}
            put[a] = c
            ops.append(O.MapUp(O.Dot(a, c), k, O.MVRegPut(O.VClock(put), int(rng.integers(1, 1000)))))
        streams.append(ops)
    exp = []
    for m, ops in zip(states, streams):
        m = m.copy()
        for op in ops:
            m.apply(op)
        exp.append(m)
    dev = lambda x: torch.from_numpy(x.view(np.int64).copy()).to("cuda:0")  # noqa: E731
    t = [dev(x) for x in (clock, ec, vclk, vval, dcl, dks)]
    tc = torch.from_numpy(cnt).to("cuda:0")
    ops = cg.map.encode_ops([[op_tuple(o) for o in s] for s in streams], A, "cuda:0")
    status = cg.map.apply_batch(*t, tc, ops, ctx=mactx).cpu().numpy()
    torch.cuda.synchronize()
    assert not (status & ~16).any(), sorted(set(status.tolist()))
    c, e, vc, vv = (to_host(x) for x in t[:4])
    dc, dk, n = to_host(t[4]), to_host(t[5]), tc.cpu().numpy()
    for s in range(N):
        if status[s] & 16:
            continue  # more concurrent values than V slots: reported, not compared
        deferred = [(dc[s, d], O.bitmap_members(dk[s, d])) for d in range(int(n[s]))]
        got = O.dense_to_map(c[s], e[s], vc[s], vv[s], deferred)
        assert got == exp[s], s
    assert (status == 0).sum() > N // 2
