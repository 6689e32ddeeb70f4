"""Seeded global inputs of the world-2 real-kernel sharding check (tests/test_gpu_dist_world2.py
and its worker): every rank and the checking parent rebuild the same arrays."""
import numpy as np

import oracle as O

# name -> (kind, G, R, W): W = row width in u64 words (2A for PNCounter, bitmap words for GSet)
LATTICES = {
    "vclock": ("vclock", 3, 301, 64),
    "gcounter": ("gcounter", 1, 1000, 256),
    "pncounter": ("pncounter", 2, 257, 2 * 40),
    "gset": ("gset", 2, 123, 17),
}
MAP_VOUT = 8


def lattice_input(name):
    kind, G, R, W = LATTICES[name]
    return O.synth_matrix(0x5EED0005 + len(name), G * R, W, 1 if kind == "gset" else 0).reshape(G, R, W)


def lww_input():
    m = O.synth_matrix(43, 3, 201, 2) % np.uint64(9)
    v = O.synth_matrix(43, 3, 201, 3) % np.uint64(2)
    return m, v


def orswot_input():
    return O.gen_orswot(99, 41, 70, 9, kmax=10)


def map_input():
    """Op-replay replicas plus 6 removes from the far future (never dominated by any clock, so they
    survive the fold and their key sets must come out of the exchange); the fold is exact for
    any input, so these need not be pre-applied to the replicas."""
    K, A = 29, 6
    maps = O.gen_map_replicas(7, 37, K, A, steps=300, p_rm=0.3, p_up=0.4)
    d = O.map_to_dense(maps, K, A, O.max_vals(maps))
    rng = np.random.default_rng(5)
    R = d["clock"].shape[0]
    rows = rng.integers(0, R, size=6).astype(np.uint64)
    clk = np.zeros((6, A), np.uint64)
    clk[np.arange(6), rng.integers(0, A, size=6)] = 10**6 + np.arange(6, dtype=np.uint64) % 3
    keys = np.zeros((6, (K + 63) // 64), np.uint64)
    for j in range(6):
        for k in rng.choice(K, size=3, replace=False):
            keys[j, k // 64] |= np.uint64(1) << np.uint64(k % 64)
    row = np.concatenate([d["def_row"].astype(np.uint64), rows])
    order = np.argsort(row, kind="stable")
    d["def_row"] = row[order]
    d["def_clock"] = np.concatenate([d["def_clock"], clk])[order]
    d["def_keys"] = np.concatenate([d["def_keys"], keys])[order]
    return d
