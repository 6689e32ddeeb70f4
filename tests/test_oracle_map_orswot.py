"""CPU: the oracle's Map<K, Orswot<M>> (round 4) — dense ingest / egress round trips (nested
deferred removes included) and the non-associativity that makes the GPU fold each key in replica
order."""
import numpy as np

import oracle as O


def _egress(d, r, K):
    vd = {}
    for k in range(K):
        lo, hi = int(d["vd_off"][r * K + k]), int(d["vd_off"][r * K + k + 1])
        vd[k] = [(d["vd_clock"][i], O.bitmap_members(d["vd_members"][i:i + 1])) for i in range(lo, hi)]
    dm = [(d["def_clock"][i], {k for k in range(K) if (int(d["def_keys"][i][k // 64]) >> (k % 64)) & 1})
          for i in range(len(d["def_row"])) if int(d["def_row"][i]) == r]
    return O.dense_to_map_orswot(d["clock"][r], d["ec"][r], d["oc"][r], d["ent"][r], vd, dm)


def test_dense_round_trip():
    maps = O.map_orswot_objects(40, 5, 6, 4, seed=3, steps=300)
    assert sum(len(e.val.deferred) for m in maps for e in m.entries.values()) > 0
    d = O.map_orswot_to_dense(maps, 5, 6, 4)
    for r, m in enumerate(maps):
        assert _egress(d, r, 5) == m
    assert d["ent"].shape == (40, 5, 6, 4)


def test_fold_not_associative():
    maps = O.map_orswot_objects(30, 4, 5, 4, seed=8, steps=300)
    differ = 0
    for t in range(30):
        idx = np.random.default_rng(t).permutation(len(maps))[:9]
        ms = [maps[i] for i in idx]
        left = O.map_fold_objects(ms)
        a, b = O.map_fold_objects(ms[:4]), O.map_fold_objects(ms[4:])
        a.merge(b)
        differ += not (a.clock == left.clock and a.entries == left.entries)
    assert differ > 0
