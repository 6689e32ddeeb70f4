"""CPU: the oracle's Map<K, GCounter> / Map<K, PNCounter> (round 4) — the counter values' merge and
forget restated from gcounter.rs:44-54 / pncounter.rs:70-82, dense ingest / egress round trips,
and the fact that makes the GPU fold each key in replica order: the Map fold with these values is
not associative on op-replay histories (a tree of partial folds differs from the left fold)."""
import numpy as np
import pytest

import oracle as O


def test_counter_forget_is_vclock_forget():
    g = O.GCounter()
    g.inner = O.VClock({0: 3, 1: 5, 2: 1})
    g.forget(O.VClock({0: 3, 1: 4, 3: 9}))  # keep x[a] iff x[a] > clock[a] (vclock.rs:95-105)
    assert g.inner == O.VClock({1: 5, 2: 1})
    c = O.PNCounter()
    c.p.inner, c.n.inner = O.VClock({0: 2}), O.VClock({0: 4, 1: 1})
    c.forget(O.VClock({0: 3}))
    assert c.p.inner == O.VClock() and c.n.inner == O.VClock({0: 4, 1: 1})


@pytest.mark.parametrize("W", [1, 2])
def test_dense_round_trip(W):
    maps = O.map_counter_objects(25, 5, 4, W, seed=21, steps=200, p_rm=0.3)
    d = O.map_counter_to_dense(maps, 5, 4, W)
    for r, m in enumerate(maps):
        b = O.dense_to_map_counter(d["clock"][r], d["ec"][r], d["val"][r])
        assert b.clock == m.clock and b.entries == m.entries
    assert d["val"].shape == (25, 5, W, 4)


@pytest.mark.parametrize("W", [1, 2])
def test_fold_not_associative(W):
    maps = O.map_counter_objects(30, 6, 5, W, seed=3 + W, steps=400, p_rm=0.3)
    differ = 0
    for t in range(30):
        idx = np.random.default_rng(t).permutation(len(maps))[:9]
        ms = [maps[i] for i in idx]
        left = O.map_fold_objects(ms)
        a, b = O.map_fold_objects(ms[:4]), O.map_fold_objects(ms[4:])
        a.merge(b)
        differ += not (a.clock == left.clock and a.entries == left.entries)
    assert differ > 0
