"""The multi-core CPU baselines of configs 3 and 4 (oracle/ref_fold.cpp oracle_orswot_fold_mt /
oracle_map_fold_mt; bench.py's c3 / c4 cpu_baseline) compute the same fold as the single-threaded
restatement: Orswot split by replica ranges then the partials merged (orswot.rs:81-149), Map<K, MVReg>
split by key ranges (map.rs:140-220 is per key given the clocks and the deferred list).  Test
infrastructure: these are baselines, never the product path."""
import numpy as np
import pytest

import oracle as O


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_orswot_fold_mt_equals_left_fold(threads):
    clock, entries, off, dcl, dmem = O.gen_orswot(11, 70, 40, 6, kmax=12, p_def=0.3)
    one = O.orswot_fold(clock, entries, off, dcl, dmem)
    mt = O.orswot_fold(clock, entries, off, dcl, dmem, threads=threads)
    assert np.array_equal(one[0], mt[0]) and np.array_equal(one[1], mt[1]) and one[2] == mt[2]
    assert one[2]  # removes survive at this shape


def test_orswot_fold_mt_synthetic_config3_shape():
    """The bench's generator (c3: crdt_synth_orswot) at a small member count, 16 threads."""
    c, e = O.synth_orswot(0x5EED0003, 300, 64, 16, 48)
    one = O.orswot_fold(c, e)
    mt = O.orswot_fold(c, e, threads=16)
    assert np.array_equal(one[0], mt[0]) and np.array_equal(one[1], mt[1]) and one[2] == mt[2]


@pytest.mark.parametrize("threads", [1, 4, 16])
def test_map_fold_mt_equals_left_fold(threads):
    seed, R, K, A, V, kmax = 0x5EED0004, 600, 96, 8, 2, 40
    rows, dcl, dks = O.synth_map_deferred(seed, R, K, A, kmax, p_def=0.3)
    d = O.synth_map(seed, R, K, A, V, kmax, deferred=(rows, dcl, dks))
    # removes from the far future on a few keys, so survivors with key sets spanning threads exist
    rng = np.random.default_rng(3)
    extra = np.zeros((6, A), np.uint64)
    extra[np.arange(6), rng.integers(0, A, 6)] = np.uint64(10**6)
    eks = np.zeros((6, (K + 63) // 64), np.uint64)
    for j in range(6):
        for k in rng.choice(K, size=5, replace=False):
            eks[j, k // 64] |= np.uint64(1) << np.uint64(k % 64)
    r2 = np.concatenate([rows, rng.integers(0, R, 6)])
    order = np.argsort(r2, kind="stable")
    r2, dc2, dk2 = r2[order], np.concatenate([dcl, extra])[order], np.concatenate([dks, eks])[order]
    one = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], r2, dc2, dk2, 4)
    mt = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], r2, dc2, dk2, 4, threads=threads)
    for i in range(5):
        assert np.array_equal(one[i], mt[i]), i
    assert one[5] == mt[5] and len(one[5]) >= 6
