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


def map_overflow_input():
    """Map input whose LAST key folds through 12 concurrent values (6 replicas x 2 concurrent
    writes by distinct actors) while every other key holds one: in a key-sharded fold with vout=8
    only the rank owning the last key sees its fold state overflow (flags bit 2), and every rank
    must rerun with the larger state together (the retry used to be rank-local)."""
    R, K, V, A = 6, 5, 2, 12
    clock = np.zeros((R, A), np.uint64)
    ec = np.zeros((R, K, A), np.uint64)
    vclk = np.zeros((R, K, V, A), np.uint64)
    vval = np.zeros((R, K, V), np.uint64)
    for r in range(R):
        for t in range(V):
            a = r * V + t
            clock[r, a] = 1
            ec[r, K - 1, a] = 1
            vclk[r, K - 1, t, a] = 1
            vval[r, K - 1, t] = 100 * r + t
        ec[r, : K - 1, 0] = clock[r, 0]  # the other keys: one write by actor 0 (replica 0 only)
        vclk[r, : K - 1, 0, 0] = clock[r, 0]
        vval[r, : K - 1, 0] = 7 * (r + 1) * (clock[r, 0] > 0)
    return dict(clock=clock, ec=ec, vclk=vclk, vval=vval, def_row=np.zeros(0, np.uint64),
                def_clock=np.zeros((0, A), np.uint64), def_keys=np.zeros((0, 1), np.uint64))


MAP_OVF_VOUT = 16


# BASELINE config 5, one GPU's shard per rank (bench.py --workload c5): VClock 1,048,576 x 1,024
C5_R, C5_A, C5_SEED = 1 << 20, 1024, 0x5EED0005
C5_COLS = np.array([0, 1, 2, 63, 64, 127, 255, 256, 511, 512, 700, 777, 1000, 1021, 1022, 1023])


def c5_expected_columns(R, row0=0):
    """The oracle's left fold of VClock::merge (oracle_vclock_fold) over rows [row0, row0 + R) of the
    config-5 synthetic input, restricted to the sampled actor columns C5_COLS (the generator is
    closed-form per (row, actor), so a column is generated without the other 1,008)."""
    r = np.arange(row0, row0 + R, dtype=np.uint64)
    idx = r[:, None] * np.uint64(C5_A) + C5_COLS.astype(np.uint64)[None, :]
    return O.vclock_fold(O.synth_values(C5_SEED, idx, 0))[0]


def adversarial_orswot(seed, R, M, A, V=6, p_def=0.3, plant=True):
    """Arbitrary states (E > C cells, repeated dots) plus deferred removes per replica; with `plant`,
    the smallest non-associative cell sequence (e, c) = (1, 1), (2, 0), (1, 2) is planted on member 0,
    actor 0 at replicas 0, R-2, R-1 (all other replicas zero there), so a fold that joins slice
    partials as a tree keeps a dot the left fold drops."""
    rng = np.random.default_rng(seed)
    clock = rng.integers(0, V, size=(R, A)).astype(np.uint64)
    entries = rng.integers(0, V, size=(R, M, A)).astype(np.uint64)
    entries[rng.random((R, M, A)) < 0.6] = 0
    if plant and R >= 3:
        clock[:, 0] = 0
        entries[:, 0, 0] = 0
        for r, (e, c) in zip((0, R - 2, R - 1), ((1, 1), (2, 0), (1, 2))):
            entries[r, 0, 0], clock[r, 0] = e, c
    Mw = (M + 63) // 64
    off, dcl, dmem = [0], [], []
    for _ in range(R):
        if rng.random() < p_def:
            rm = rng.integers(0, V + 1, size=A).astype(np.uint64)
            if plant:
                rm[0] = 0  # removes never touch the planted cell
            dcl.append(rm)
            bits = np.zeros(Mw, np.uint64)
            for m in rng.choice(M, size=min(M, 3), replace=False):
                if not plant or m != 0:
                    bits[m // 64] |= np.uint64(1) << np.uint64(m % 64)
            dmem.append(bits)
        off.append(len(dcl))
    return (clock, entries, np.array(off, np.uint64), np.array(dcl, np.uint64).reshape(-1, A),
            np.array(dmem, np.uint64).reshape(-1, Mw))


def orswot_any_input():
    """World-2 Orswot input outside the reference invariants (see adversarial_orswot)."""
    return adversarial_orswot(0x5EED00A1, 600, 11, 8)
