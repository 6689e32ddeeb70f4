"""Batched Orswot CmRDT::apply (crdt_orswot_apply_batch) vs the oracle's one-by-one apply
(orswot.rs:55-79, apply_rm :230-250, apply_deferred :281-286).

Inputs: the reference's own KAT scripts with every Orswot op routed through the kernel, op-replay
streams built with the reference's ctx API (test/orswot.rs:15-31 style: one actor per origin,
out-of-order delivery so removes defer), and arbitrary ops on arbitrary states (the kernel
claims exactness for any input, not only for states the reference can reach)."""
import numpy as np
import pytest
import torch

import kat_runner as K
import oracle as O
from gpu_util import to_dev, to_host
from orswot_apply_util import (arbitrary_case, dense_states, map_orswot, op_tuple, oracle_streams,
                               replay_streams, to_object)

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


@pytest.fixture(scope="module", params=["alane=1", "alane=1,oameta=0", "alane=1,oastg=1", "alane=1,oastg=1,oameta=0", "alane=1,oapf=1", "alane=1,ohpf=1", "alane=0"])
def actx(request):
    """Both kernels: 16 lanes per state (alane=1, the default for A <= 64; its batch's first two Rm
    clock rows staged in LDS by LDS-DMA for even A with oastg=1, opt-in) and one wave per state (alane=0,
    every A); shapes with A > 64 take the wave kernel in both modes."""
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    ctx = cg.Context(0)
    ctx.tune(request.param)
    yield ctx
    ctx.close()


def gpu_apply_streams(ctx, states, streams, M, A, Dcap=None):
    """Apply streams[s] to a copy of states[s] for every s in one batched call; returns the
    resulting oracle objects and the status array."""
    if Dcap is None:
        Dcap = max(1, max(len(o.deferred) for o in states) + max(
            sum(1 for op in ops if isinstance(op, O.OrswotRm)) for ops in streams))
    clock, entries, dcl, dmb, cnt = dense_states(states, M, A, Dcap)
    tc, te, tdc, tdm = to_dev(clock), to_dev(entries), to_dev(dcl), to_dev(dmb)
    tcnt = torch.from_numpy(cnt).cuda()
    ops = cg.orswot.encode_ops([[op_tuple(op) for op in ops] for ops in streams], A, "cuda:0")
    status = cg.orswot.apply_batch(tc, te, tdc, tdm, tcnt, ops, ctx=ctx)
    torch.cuda.synchronize()
    c, e, d, dm = to_host(tc), to_host(te), to_host(tdc), to_host(tdm)
    n = tcnt.cpu().numpy()
    return [to_object(c, e, d, dm, n, s) for s in range(len(states))], status.cpu().numpy()


# ---- the reference's KATs with Orswot apply on the GPU ------------------------------------------
def gpu_apply_hook(ctx):
    """Route one Orswot op through crdt_orswot_apply_batch: intern the state's and the op's
    actors / members (KAT ids are strings and ints), apply, map the result back in place."""
    def hook(v, op):
        actors, members = cg.intern.Index(), cg.intern.Index()
        iv = map_orswot(v, actors.intern, members.intern)
        if isinstance(op, O.OrswotAdd):
            iop = O.OrswotAdd(O.Dot(actors.intern(op.dot.actor), op.dot.counter), [members.intern(m) for m in op.members])
        else:
            iop = O.OrswotRm(O.VClock({actors.intern(a): c for a, c in op.clock.dots.items()}),
                             [members.intern(m) for m in op.members])
        (res,), status = gpu_apply_streams(ctx, [iv], [[iop]], max(1, len(members)), max(1, len(actors)))
        assert status[0] == 0
        back = map_orswot(res, lambda a: actors.ids[a], lambda m: members.ids[m])
        v.clock, v.entries, v.deferred = back.clock, back.entries, back.deferred
    return hook


APPLY_CASES = [c for c in K.load_cases("kat_orswot.json")
               if any(s[0] in ("add", "rm", "rm_clock", "add_ctx", "rm_ctx") for s in c["steps"])]


@pytest.mark.parametrize("case", APPLY_CASES, ids=[c["name"] for c in APPLY_CASES])
def test_kat_orswot_apply_gpu(actx, case):
    K.run_case(case, apply_hook=gpu_apply_hook(actx))


# ---- op replay (ctx API, one actor per origin, out-of-order delivery) ---------------------------
@pytest.mark.parametrize("seed,n_states,n_origins,M,n_ops", [
    (1, 64, 4, 12, 60), (2, 200, 8, 40, 150), (3, 16, 64, 200, 400), (4, 100, 3, 5, 100)])
def test_orswot_apply_replay(actx, seed, n_states, n_origins, M, n_ops):
    streams = replay_streams(seed, n_states, n_origins, M, n_ops)
    states = [O.Orswot() for _ in streams]
    got, status = gpu_apply_streams(actx, states, streams, M, n_origins)
    exp = oracle_streams(states, streams)
    assert (status == 0).all()
    assert sum(len(o.deferred) for o in exp) > 0 or seed == 4  # the replay exercises deferral
    for s, (g, e) in enumerate(zip(got, exp)):
        assert g == e, f"state {s}: {g} != {e}"


# ---- arbitrary states and ops ------------------------------------------------------------------
@pytest.mark.parametrize("seed,N,M,A", [(5, 40, 16, 8), (6, 24, 70, 65), (7, 8, 130, 256), (8, 30, 3, 1)])
def test_orswot_apply_arbitrary(actx, seed, N, M, A):
    states, streams = arbitrary_case(seed, N, M, A)
    got, status = gpu_apply_streams(actx, states, streams, M, A)
    exp = oracle_streams(states, streams)
    assert (status == 0).all()
    for s, (g, e) in enumerate(zip(got, exp)):
        assert g == e, f"state {s}"


def test_orswot_apply_overflow_and_bad_ops(actx):
    A, M = 4, 8
    st = [O.Orswot(), O.Orswot(), O.Orswot()]
    fut1 = O.OrswotRm(O.VClock({0: 5}), [1])
    fut2 = O.OrswotRm(O.VClock({1: 5}), [2])
    add = O.OrswotAdd(O.Dot(2, 1), [3])
    streams = [[fut1, fut2, add], [add, fut1, fut1], [add]]
    got, status = gpu_apply_streams(actx, st, streams, M, A, Dcap=1)
    assert status[0] & 1 and status[1] == 0 and status[2] == 0  # state 0 needs 2 deferred slots
    exp = oracle_streams(st, streams)
    assert got[1] == exp[1] and got[2] == exp[2]
    # an out-of-range member is skipped and flagged; the rest of the op still applies
    bad = O.OrswotAdd(O.Dot(0, 1), [2, 99])
    got, status = gpu_apply_streams(actx, [O.Orswot()], [[bad]], M, A, Dcap=1)
    assert status[0] == 2
    assert set(got[0].entries) == {2} and got[0].clock.dots == {0: 1}


def test_orswot_apply_malformed_headers(actx):
    """Ops with kind > 1, a reversed member range or a member range ending at or beyond 2^32 are
    skipped and flagged (status bit 2) without touching memory; the rest of the stream applies."""
    A, M, Dcap = 4, 8, 2
    add1, add2 = O.OrswotAdd(O.Dot(0, 1), [2]), O.OrswotAdd(O.Dot(1, 1), [3])
    rm = O.OrswotRm(O.VClock({0: 1}), [4])
    streams = [[add1, add2], [add1, rm], [add1, add2]]
    st = [O.Orswot() for _ in streams]
    clock, entries, dcl, dmb, cnt = dense_states(st, M, A, Dcap)
    tc, te, tdc, tdm = to_dev(clock), to_dev(entries), to_dev(dcl), to_dev(dmb)
    tcnt = torch.from_numpy(cnt).cuda()
    ops = cg.orswot.encode_ops([[op_tuple(op) for op in ops] for ops in streams], A, "cuda:0")
    ops.mem_off[2] = 1 << 32           # state 0's last op (op 1): member range reaches 2^32
    ops.kind[2] = 2                    # state 1's first op: no such kind
    ops.mem_off[6] = ops.mem_off[5] - 1  # state 2's last op (op 5): reversed range
    status = cg.orswot.apply_batch(tc, te, tdc, tdm, tcnt, ops, ctx=actx).cpu().numpy()
    torch.cuda.synchronize()
    assert status.tolist() == [2, 2, 2]
    got = [to_object(to_host(tc), to_host(te), to_host(tdc), to_host(tdm), tcnt.cpu().numpy(), s) for s in range(3)]
    exp = oracle_streams(st, [[add1], [rm], [add1]])
    assert got == exp


def test_orswot_apply_member_range_past_buffer(actx):
    """A member range that runs past the n_mem entries of `mem` is malformed (status bit 1): the
    op is skipped without reading past the buffer, the rest of the stream applies."""
    A, M, Dcap = 4, 8, 2
    add1, add2 = O.OrswotAdd(O.Dot(0, 1), [2]), O.OrswotAdd(O.Dot(1, 1), [3, 5])
    rm = O.OrswotRm(O.VClock({0: 1}), [2])
    streams = [[add1, rm], [add1, add2]]
    st = [O.Orswot() for _ in streams]
    clock, entries, dcl, dmb, cnt = dense_states(st, M, A, Dcap)
    tc, te, tdc, tdm = to_dev(clock), to_dev(entries), to_dev(dcl), to_dev(dmb)
    tcnt = torch.from_numpy(cnt).cuda()
    ops = cg.orswot.encode_ops([[op_tuple(op) for op in ops] for ops in streams], A, "cuda:0")
    n_mem = ops.mem.shape[0]
    ops.mem_off[2] = n_mem + 1         # op 1 (state 0's Rm) ends one past mem; op 2 is then reversed
    ops.mem_off[4] = n_mem + 4096      # op 3 (state 1's add2, the last op) ends far past mem
    status = cg.orswot.apply_batch(tc, te, tdc, tdm, tcnt, ops, ctx=actx).cpu().numpy()
    torch.cuda.synchronize()
    assert status.tolist() == [2, 2]
    got = [to_object(to_host(tc), to_host(te), to_host(tdc), to_host(tdm), tcnt.cpu().numpy(), s) for s in range(2)]
    assert got == oracle_streams(st, [[add1], []])


def test_orswot_apply_empty(actx):
    st = [O.Orswot() for _ in range(5)]
    got, status = gpu_apply_streams(actx, st, [[] for _ in st], 4, 2, Dcap=1)
    assert (status == 0).all() and all(g == O.Orswot() for g in got)


@pytest.mark.parametrize("N,T,M,A", [(512, 64, 300, 64), (64, 200, 40, 256), (300, 32, 1000, 17),
                                     (8, 64, 300000, 4), (6, 64, 600000, 4)])
def test_orswot_apply_synth_streams(actx, N, T, M, A):
    """The bench's device-generated streams vs the C++ twin (std containers), every state.  The
    last two shapes have member bitmaps so wide that one / no deferred slot fits the 64 KiB of LDS:
    the rest live in the states' HBM slots (no capacity error)."""
    ops = cg.synth.orswot_op_streams(N, T, M, A, seed=N + T, device="cuda:0")
    Dcap = 16
    clock = torch.zeros((N, A), dtype=torch.int64, device="cuda:0")
    entries = torch.zeros((N, M, A), dtype=torch.int64, device="cuda:0")
    dcl = torch.zeros((N, Dcap, A), dtype=torch.int64, device="cuda:0")
    dmb = torch.zeros((N, Dcap, (M + 63) // 64), dtype=torch.int64, device="cuda:0")
    cnt = torch.zeros(N, dtype=torch.int32, device="cuda:0")
    status = cg.orswot.apply_batch(clock, entries, dcl, dmb, cnt, ops, ctx=actx)
    torch.cuda.synchronize()
    arr = [t.cpu().numpy() for t in ops]
    oc, oe, ond, _ = O.orswot_apply_streams(N, M, A, *arr)
    assert (status.cpu().numpy() == 0).all()
    np.testing.assert_array_equal(to_host(clock), oc)
    np.testing.assert_array_equal(to_host(entries), oe)
    np.testing.assert_array_equal(cnt.cpu().numpy(), ond.astype(np.int32))
    assert ond.sum() > 0


@pytest.mark.parametrize("hot", [0, 1, 3])
def test_orswot_apply_deferred_spill(hot):
    """Deferred slots beyond the LDS-resident ones live in the state's HBM slots (CRDT_TUNE hot=N):
    the same results with none, one or three slots in LDS."""
    ctx = cg.Context(0)
    ctx.tune(f"hot={hot},alane=0")  # (LDS-resident slots: the wave-per-state kernel)
    try:
        states, streams = arbitrary_case(9 + hot, 24, 40, 16, max_ops=60)
        got, status = gpu_apply_streams(ctx, states, streams, 40, 16)
        exp = oracle_streams(states, streams)
        assert (status == 0).all()
        assert max(len(e.deferred) for e in exp) > hot  # some state really spills to HBM
        for s, (g, e) in enumerate(zip(got, exp)):
            assert g == e, s
    finally:
        ctx.close()


@pytest.mark.parametrize("mode", ["lub2", "merge_batch"])
@pytest.mark.parametrize("case", APPLY_CASES, ids=[c["name"] for c in APPLY_CASES])
def test_kat_orswot_apply_and_merge_gpu(actx, case, mode):
    """The reference's Orswot KATs (test/orswot.rs, orswot.rs:294-394) with EVERY apply and EVERY
    merge on the GPU (crdt_orswot_apply_batch; crdt_orswot_lub_many of the pair or the in-place
    crdt_orswot_merge_batch)."""
    from test_gpu_kat import gpu_merge
    K.run_case(case, merge_hook=lambda d, s, k: gpu_merge(d, s, k, mode), apply_hook=gpu_apply_hook(actx))
