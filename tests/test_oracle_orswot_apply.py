"""CPU: the dense Orswot apply restatement (oracle.dense_orswot_apply — the algorithm the
crdt_orswot_apply_batch kernel runs per state) equals the reference-shaped Orswot.apply
(orswot.rs:55-79, :230-250, :281-286) on op-replay streams, arbitrary inputs and the KATs."""
import numpy as np
import pytest

import kat_runner as K
import oracle as O
from orswot_apply_util import (arbitrary_case, dense_states, map_orswot, op_tuple, oracle_streams,
                               replay_streams, to_object)


def dense_apply_streams(states, streams, M, A, Dcap=None):
    if Dcap is None:
        Dcap = max(1, max(len(o.deferred) for o in states) + max(
            sum(1 for op in ops if isinstance(op, O.OrswotRm)) for ops in streams))
    clock, entries, dcl, dmb, cnt = dense_states(states, M, A, Dcap)
    status = np.zeros(len(states), np.int32)
    for s, ops in enumerate(streams):
        enc = []
        for op in ops:
            t = op_tuple(op)
            if t[0] == "rm":
                row = np.zeros(A, np.uint64)
                for a, v in t[1].items():
                    row[a] = v
                t = ("rm", row, t[2])
            enc.append(t)
        cnt[s], status[s] = O.dense_orswot_apply(clock[s], entries[s], dcl[s], dmb[s], int(cnt[s]), enc)
    return [to_object(clock, entries, dcl, dmb, cnt, s) for s in range(len(states))], status


@pytest.mark.parametrize("seed,n_states,n_origins,M,n_ops", [(1, 24, 4, 12, 60), (2, 20, 8, 40, 150)])
def test_dense_apply_replay(seed, n_states, n_origins, M, n_ops):
    streams = replay_streams(seed, n_states, n_origins, M, n_ops)
    states = [O.Orswot() for _ in streams]
    got, status = dense_apply_streams(states, streams, M, n_origins)
    exp = oracle_streams(states, streams)
    assert (status == 0).all()
    assert sum(len(o.deferred) for o in exp) > 0
    assert got == exp


@pytest.mark.parametrize("seed,N,M,A", [(5, 20, 16, 8), (6, 10, 70, 65), (8, 20, 3, 1)])
def test_dense_apply_arbitrary(seed, N, M, A):
    states, streams = arbitrary_case(seed, N, M, A)
    got, status = dense_apply_streams(states, streams, M, A)
    assert (status == 0).all()
    assert got == oracle_streams(states, streams)


def _dense_hook(v, op):
    from crdts_gpu.intern import Index
    actors, members = Index(), Index()
    iv = map_orswot(v, actors.intern, members.intern)
    if isinstance(op, O.OrswotAdd):
        iop = O.OrswotAdd(O.Dot(actors.intern(op.dot.actor), op.dot.counter), [members.intern(m) for m in op.members])
    else:
        iop = O.OrswotRm(O.VClock({actors.intern(a): c for a, c in op.clock.dots.items()}),
                         [members.intern(m) for m in op.members])
    (res,), status = dense_apply_streams([iv], [[iop]], max(1, len(members)), max(1, len(actors)))
    assert status[0] == 0
    back = map_orswot(res, lambda a: actors.ids[a], lambda m: members.ids[m])
    v.clock, v.entries, v.deferred = back.clock, back.entries, back.deferred


APPLY_CASES = [c for c in K.load_cases("kat_orswot.json")
               if any(s[0] in ("add", "rm", "rm_clock", "add_ctx", "rm_ctx") for s in c["steps"])]


@pytest.mark.parametrize("case", APPLY_CASES, ids=[c["name"] for c in APPLY_CASES])
def test_kat_dense_apply(case):
    K.run_case(case, apply_hook=_dense_hook)


def test_dense_apply_overflow():
    st = [O.Orswot()]
    ops = [O.OrswotRm(O.VClock({0: 5}), [1]), O.OrswotRm(O.VClock({1: 5}), [2])]
    _, status = dense_apply_streams(st, [ops], 8, 4, Dcap=1)
    assert status[0] == 1
