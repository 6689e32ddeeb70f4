"""The dense Map<K, MVReg> fold (what the GPU kernel implements, oracle.dense_map_fold) equals
the reference fold restated over map-based states — the Python object twin (map.rs:140-220,
mvreg.rs:88-128) and the C++ twin (oracle/ref_fold.cpp oracle_map_fold) — on op-replay
replicas (realistic, with deferred removes) and on arbitrary dense states (exactness does
not rely on any invariant)."""
import numpy as np
import pytest

import oracle as O


def _fold_all(d, Vout):
    py = O.dense_map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                          d["def_keys"], Vout)
    cc = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"],
                    d["def_keys"], Vout)
    return py, cc


def _same(py, cc):
    for x, y, nm in zip(py[:5], cc[:5], ("clock", "ec", "vclk", "vval", "nval")):
        assert np.array_equal(np.asarray(x), np.asarray(y)), nm
    assert py[5] == cc[5], "deferred"


@pytest.mark.parametrize("seed", range(80))
def test_dense_fold_matches_object_fold(seed):
    rng = np.random.default_rng(seed)
    K, A = int(rng.integers(1, 12)), int(rng.integers(1, 6))
    R = int(rng.integers(1, 14))
    p_rm = float(rng.choice([0.15, 0.3, 0.45]))
    maps = O.gen_map_replicas(seed, R, K, A, steps=int(rng.integers(10, 160)), p_rm=p_rm,
                              p_up=0.7 - p_rm)
    V = O.max_vals(maps)
    d = O.map_to_dense(maps, K, A, V)
    acc = O.map_fold_objects(maps)
    Vout = max(V, O.max_vals([acc]))
    py, cc = _fold_all(d, Vout)
    _same(py, cc)
    # compare with the object fold in dense form (ordered vals: MVReg's own PartialEq panics
    # on duplicate (clock, val) pairs, mvreg.rs:72, which out-of-order op replay can produce)
    ref = O.map_to_dense([acc], K, A, Vout)
    assert np.array_equal(py[0], ref["clock"][0])
    assert np.array_equal(py[1], ref["ec"][0])
    assert np.array_equal(py[2], ref["vclk"][0])
    assert np.array_equal(py[3], ref["vval"][0])
    assert py[5] == {(tuple(int(x) for x in c), O.bitmap_members(b))
                     for c, b in zip(ref["def_clock"], ref["def_keys"])}


def _random_dense(rng, R, K, A, V, cmax):
    clock = rng.integers(0, cmax, size=(R, A)).astype(np.uint64)
    ec = rng.integers(0, cmax, size=(R, K, A)).astype(np.uint64)
    ec[rng.random((R, K)) < 0.3] = 0
    nv = rng.integers(0, V + 1, size=(R, K))
    vclk = rng.integers(0, cmax, size=(R, K, V, A)).astype(np.uint64)
    vclk[rng.random((R, K, V, A)) < 0.4] = 0
    for s in range(V):
        vclk[:, :, s][nv <= s] = 0
    # keep used slots packed first (an emptied middle slot would shift the Vec order)
    for r in range(R):
        for k in range(K):
            rows = [vclk[r, k, s].copy() for s in range(V) if vclk[r, k, s].any()]
            vclk[r, k] = 0
            for s, row in enumerate(rows):
                vclk[r, k, s] = row
    vval = rng.integers(0, 5, size=(R, K, V)).astype(np.uint64)
    D = int(rng.integers(0, R + 1))
    def_row = np.sort(rng.integers(0, R, size=D)).astype(np.uint64)
    def_clock = rng.integers(0, cmax + 2, size=(D, A)).astype(np.uint64)
    def_keys = np.zeros((D, (K + 63) // 64), np.uint64)
    for d in range(D):
        for k in rng.choice(K, size=int(rng.integers(1, K + 1)), replace=False):
            def_keys[d, k // 64] |= np.uint64(1) << np.uint64(k % 64)
    return dict(clock=clock, ec=ec, vclk=vclk, vval=vval, def_row=def_row, def_clock=def_clock,
                def_keys=def_keys)


@pytest.mark.parametrize("seed", range(40))
def test_dense_fold_arbitrary_states(seed):
    rng = np.random.default_rng(100 + seed)
    R, K, A, V = (int(rng.integers(1, 10)), int(rng.integers(1, 8)), int(rng.integers(1, 5)),
                  int(rng.integers(1, 4)))
    d = _random_dense(rng, R, K, A, V, cmax=int(rng.choice([3, 6, 1000])))
    py, cc = _fold_all(d, Vout=R * V + 1)
    _same(py, cc)


def test_synth_map_deferred_twins():
    """crdts_gpu.synth.map_deferred (vectorised, what the product-side generator uploads) and
    oracle.synth_map_deferred (loop restatement) build the same deferred lists."""
    import crdts_gpu.synth as S
    for seed, R, K, A, kmax in [(1, 300, 64, 8, 40), (2, 100, 10, 1, 5), (3, 200, 33, 2, 9),
                                (4, 500, 1024, 32, 256)]:
        a = S.map_deferred(seed, R, K, A, kmax, p_def=0.2)
        b = O.synth_map_deferred(seed, R, K, A, kmax, p_def=0.2)
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x), np.asarray(y))


@pytest.mark.parametrize("seed,R,K,A,kmax", [(5, 120, 64, 8, 40), (6, 80, 17, 3, 12), (7, 60, 9, 1, 20)])
def test_synth_map_converges_to_max_prefix(seed, R, K, A, kmax):
    """Without deferred removes every synthetic replica is a causally closed state of one op
    history, so the reference fold equals the state at the max prefix (as MVReg sets)."""
    d = O.synth_map(seed, R, K, A, 2, kmax)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], Vout=4)
    cm = d["clock"].max(0)
    top = O.synth_map(seed, 1, K, A, 2, kmax, clock_override=cm[None])
    assert np.array_equal(exp[1], top["ec"][0])
    for k in range(K):
        a = {(tuple(exp[2][k, s]), int(exp[3][k, s])) for s in range(4) if exp[2][k, s].any()}
        b = {(tuple(top["vclk"][0, k, s]), int(top["vval"][0, k, s])) for s in range(2) if top["vclk"][0, k, s].any()}
        assert a == b


@pytest.mark.parametrize("seed", range(4))
def test_synth_map_with_deferred_dense_fold(seed):
    R, K, A, kmax = 150, 40, 6, 30
    dfr = O.synth_map_deferred(seed, R, K, A, kmax, p_def=0.3)
    d = O.synth_map(seed, R, K, A, 2, kmax, deferred=dfr)
    py = O.dense_map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], dfr[0], dfr[1], dfr[2], 4)
    cc = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], dfr[0], dfr[1], dfr[2], 4)
    _same(py, cc)
