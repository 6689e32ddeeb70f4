"""Characterisation (oracle only): Map<K, MVReg>::merge is NOT associative on realistic op-replay
histories — folding consecutive slices and then the slice results differs from the left fold.
This is why csrc/map.hip computes the exact per-key left fold instead of a tree (DESIGN.md
§3.1).  Reference semantics: oracle.Map (map.rs:140-220, mvreg.rs:112-128)."""
import numpy as np
import pytest

import oracle as O


def _copies(ms):
    return [m.copy() for m in ms]


def test_slice_then_fold_differs_from_left_fold():
    differ = 0
    for seed in range(40):
        rng = np.random.default_rng(seed)
        K, A = int(rng.integers(1, 20)), int(rng.integers(1, 7))
        R = int(rng.integers(2, 40))
        p_rm = float(rng.choice([0.15, 0.3, 0.45]))
        maps = O.gen_map_replicas(seed, R, K, A, steps=int(rng.integers(20, 300)), p_rm=p_rm,
                                  p_up=0.7 - p_rm)
        left = O.map_fold_objects(_copies(maps))
        S = int(rng.integers(2, 6))
        L = -(-R // S)
        parts = [O.map_fold_objects(_copies(maps[i:i + L])) for i in range(0, R, L)]
        if O.map_fold_objects(parts) != left:
            differ += 1
    assert differ >= 10, differ  # 179 of 300 histories in the measurement quoted in DESIGN.md


def _sig(m):
    """Structural signature incl. the MVReg Vec order (the oracle's __eq__ is order-free)."""
    return (tuple(sorted(m.clock.dots.items())),
            tuple((k, tuple(sorted(e.clock.dots.items())),
                   tuple((tuple(sorted(c.dots.items())), v) for c, v in e.val.vals))
                  for k, e in sorted(m.entries.items())),
            tuple(sorted((tuple(sorted(c.dots.items())), tuple(sorted(ks))) for c, ks in m.deferred.items())))


@pytest.mark.parametrize("seed", range(12))
def test_fold_continues_from_its_prefix_result(seed):
    """The identity the streamed host-memory Map fold rests on (csrc/host_stage.hip
    map_lub_host_stream): fold(r_0..r_{n-1}) == fold(acc, r_k..r_{n-1}) with acc = fold(r_0..r_{k-1}),
    i.e. Map::new().merge(acc) == acc for a fold result, at every cut, MVReg Vec order included
    (map.rs:140-220, mvreg.rs:112-128)."""
    rng = np.random.default_rng(seed)
    maps = O.gen_map_replicas(seed, int(rng.integers(4, 24)), 9, 5, steps=200, p_rm=0.3, p_up=0.4)
    full = O.Map()
    for m in maps:
        full.merge(m.copy())
    for cut in range(1, len(maps)):
        acc = O.Map()
        for m in maps[:cut]:
            acc.merge(m.copy())
        cont = O.Map()
        cont.merge(acc.copy())
        for m in maps[cut:]:
            cont.merge(m.copy())
        assert _sig(cont) == _sig(full), cut
