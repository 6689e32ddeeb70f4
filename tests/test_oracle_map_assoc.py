"""Characterisation (oracle only): Map<K, MVReg>::merge is NOT associative on realistic op-replay
histories — folding consecutive slices and then the slice results differs from the left fold.
This is why csrc/map.hip computes the exact per-key left fold instead of a tree (DESIGN.md
§3.1).  Reference semantics: oracle.Map (map.rs:140-220, mvreg.rs:112-128)."""
import numpy as np

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
