"""CPU model of the counter-Map whole-chunk skip (csrc/map_counter.hip, SPL > 0, round 5).

The kernel skips a 16-step chunk when every step passes a no-change test evaluated against the state
at the chunk's start (entry clock e, value rows v_w, clock C0).  This restates that test in numpy and
checks it against the exact per-step join of the same kernel (the branch-free form of
map.rs:142-210 with the counter values' merge / forget, gcounter.rs:44-54, pncounter.rs:70-82):
whenever the test passes for a step, the join leaves (entry clock, value) unchanged — for random
small-valued states (equalities and zeros everywhere), for clocks C >= C0 (C only grows inside a
chunk), and on the config-4 generator's replicas, where it must also skip almost every chunk."""
import numpy as np
import pytest

import oracle as O

MAXU = np.uint64(0xFFFFFFFFFFFFFFFF)
Z = np.uint64(0)
ONE = np.uint64(1)


def fg(x, c):
    return np.where(x > c, x, Z)


def exact_join(C, e, v, c2, e2, v2):
    """One step's entry join + value merge / forget (before the step's removes), per lane word;
    arrays (..., A) with v / v2 (..., W, A).  Presence votes over the last axis."""
    p1 = e.any(-1, keepdims=True)
    p2 = e2.any(-1, keepdims=True)
    en = np.where(e == e2, e, np.maximum(fg(e2, C), fg(e, c2)))
    y = np.where(p1, np.where(p2, np.maximum(e, e2), c2), C)
    x = fg(y, en)
    a1 = np.where(p1[..., None, :], v, Z)
    a2 = np.where(p2[..., None, :], v2, Z)
    vn = fg(np.maximum(a1, a2), x[..., None, :])
    return en, vn


def chunk_test(C0, e, v, c2, e2, v2):
    """The kernel's per-step verdict (test_chunk in map_counter.hip) against the chunk-start state."""
    p1 = e.any(-1)
    p2 = e2.any(-1)
    em1 = np.where(e > 0, e - ONE, Z)
    TE = np.where(e > 0, em1, MAXU)
    TB = np.maximum(C0, em1)
    TVw = np.where(v == 0, MAXU, np.maximum(e[..., None, :], np.where(v > 0, v - ONE, Z)))
    TV = TVw.min(-2)
    TN = np.minimum(TE, TV)
    x = np.where(e2 > e, e2, Z)
    B = np.where(v == 0, x[..., None, :], v)
    cb = ((e2 == e) | ((c2 <= TE) & (e2 <= TB))) & (e2 <= TV) & (v2 <= B).all(-2)
    co = c2 <= TN
    ok_p1 = np.where(p2, cb.all(-1), co.all(-1))
    ok_p0 = (e2 <= C0).all(-1)
    return np.where(p1, ok_p1, ok_p0)


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("cmax,seed", [(2, 1), (3, 2), (6, 3), (40, 4)])
def test_chunk_test_is_sound_on_random_states(W, cmax, seed):
    rng = np.random.default_rng(seed)
    N, A = 200000, 3
    r = lambda p=0.6: (rng.integers(0, cmax + 1, size=(N, A)) * (rng.random((N, A)) < p)).astype(np.uint64)  # noqa: E731
    C0, e, c2, e2 = r(0.9), r(), r(0.9), r()
    v = (rng.integers(0, cmax + 1, size=(N, W, A)) * (rng.random((N, W, A)) < 0.6)).astype(np.uint64)
    v2 = (rng.integers(0, cmax + 1, size=(N, W, A)) * (rng.random((N, W, A)) < 0.6)).astype(np.uint64)
    # the state at the step: the chunk-start state (unchanged so far), a clock C >= C0
    C = np.maximum(C0, r(0.3))
    ok = chunk_test(C0, e, v, c2, e2, v2)
    en, vn = exact_join(C, e, v, c2, e2, v2)
    p1 = e.any(-1)
    # "unchanged": the entry clock, and the value while the entry is present (a stale value behind an
    # empty clock is never read: the kernel masks it by the presence vote)
    same_e = (en == e).all(-1)
    same_v = np.where(p1, (vn == v).all((-1, -2)), True)
    assert ok.any() and (~ok).any()
    bad = ok & ~(same_e & same_v)
    assert not bad.any(), np.flatnonzero(bad)[:5]


@pytest.mark.parametrize("W", [1, 2])
def test_chunk_test_skips_the_config4_generator(W):
    """On config-4-shaped replicas (the counter bench's input: the generator's value clocks as counter
    rows) the test is exact enough that only chunks where the state changes are run step by step."""
    R, K, A, kmax, seed = 4096, 1024, 32, 256, 0x5EED0004
    keys = np.array([3, 97, 500])
    dfr = O.synth_map_deferred(seed, R, K, A, kmax, p_def=0.1)
    d = O.synth_map(seed, R, K, A, 2, kmax, keys=keys, deferred=dfr)
    for ki in range(len(keys)):
        C = np.zeros(A, np.uint64)
        e = np.zeros(A, np.uint64)
        v = np.zeros((W, A), np.uint64)
        changed, passed = np.zeros(R, bool), np.zeros(R, bool)
        for r in range(R):
            if r % 16 == 0:
                C0, e0, v0 = C.copy(), e.copy(), v.copy()
            c2, e2, v2 = d["clock"][r], d["ec"][r, ki], d["vclk"][r, ki, :W]
            passed[r] = chunk_test(C0, e0, v0, c2, e2, v2)
            en, vn = exact_join(C, e, v, c2, e2, v2)
            p1 = e.any()
            changed[r] = not (np.array_equal(en, e) and (not p1 or np.array_equal(vn, v)))
            e, v, C = en, vn, np.maximum(C, c2)
        ch_pass = passed.reshape(-1, 16).all(1)
        ch_changed = changed.reshape(-1, 16).any(1)
        assert not (ch_pass & ch_changed).any()
        assert (~ch_pass).sum() <= ch_changed.sum() + 2, ((~ch_pass).sum(), ch_changed.sum())


# ---- Map<K, Orswot<M>> (csrc/map_orswot.hip, SPL > 0) ------------------------------------------------
def orswot_exact_step(C, e, oc, E, D, c2, e2, o2, E2):
    """One step of the Map<K, Orswot> fold without removes in the step (the chunk test's scope): the
    entry join, Orswot::merge (dot-survival join, held removes re-applied, oc |= o2, live re-test;
    orswot.rs:81-149) when both hold the key, the replica's Orswot when only it does, then the value
    forget by the case's clock (Causal::forget, orswot.rs:150-183).  Single state; D: list of
    (rm row, member mask).  Returns (e', oc', E', D')."""
    p1, p2 = e.any(), e2.any()
    en = np.where(e == e2, e, np.maximum(fg(e2, C), fg(e, c2)))
    if not en.any():
        return en, oc, E, D
    y = (np.maximum(e, e2) if p2 else c2) if p1 else C
    X = fg(y, en)
    if p1 and p2:
        E = np.where(E == E2, E, np.maximum(fg(E2, oc[None]), fg(E, o2[None])))
        for rm, msk in D:
            for m in range(E.shape[0]):
                if (msk >> m) & 1:
                    E[m] = fg(E[m], rm)
        oc = np.maximum(oc, o2)
        D = [(rm, msk) for rm, msk in D if (rm > oc).any()]
    elif p2:
        E, oc, D = E2.copy(), o2.copy(), []
    if X.any():  # Orswot::forget
        oc = fg(oc, X)
        E = fg(E, X[None])
        out = []
        for rm, msk in D:
            r2 = fg(rm, X)
            if not r2.any():
                continue
            hit = [i for i, (x, _) in enumerate(out) if np.array_equal(x, r2)]
            if hit:
                out[hit[0]] = (r2, msk)
            else:
                out.append((r2, msk))
        D = out
    return en, oc, E, D


def orswot_chunk_test(C0, e, oc, E, D, c2, e2, o2, E2):
    """map_orswot.hip test_chunk's per-step verdict (the state normalized: held removes applied)."""
    if any(not (rm > oc).any() for rm, _ in D):
        return False
    if not e.any():
        return bool((e2 <= C0).all())
    em1 = np.where(e > 0, e - ONE, Z)
    TE = np.where(e > 0, em1, MAXU)
    TB = np.maximum(C0, em1)
    tv = lambda v: np.where(v == 0, MAXU, np.maximum(e, np.where(v > 0, v - ONE, Z)))  # noqa: E731
    TX = tv(oc)
    for m in range(E.shape[0]):
        TX = np.minimum(TX, tv(E[m]))
    for rm, _ in D:
        TX = np.minimum(TX, tv(rm))
    if e2.any():
        TEm = np.where(E > 0, E - ONE, MAXU)
        cb = ((e2 == e) | ((c2 <= TE) & (e2 <= TB))) & (e2 <= TX) & (o2 <= oc)
        cb &= ((E2 == E) | ((E2 <= oc[None]) & (o2[None] <= TEm))).all(0)
        return bool(cb.all())
    return bool((c2 <= np.minimum(TE, TX)).all())


@pytest.mark.parametrize("cmax,seed", [(2, 5), (3, 6), (5, 7)])
def test_orswot_chunk_test_is_sound_on_random_states(cmax, seed):
    rng = np.random.default_rng(seed)
    A, MT = 3, 3
    n_pass = 0
    for _ in range(30000):
        r = lambda p=0.6, shape=(A,): (rng.integers(0, cmax + 1, size=shape) * (rng.random(shape) < p)).astype(np.uint64)  # noqa: E731
        C0, e, oc, c2, e2, o2 = r(0.9), r(), r(0.8), r(0.9), r(), r(0.8)
        E, E2 = r(0.5, (MT, A)), r(0.5, (MT, A))
        D = []
        for _ in range(int(rng.integers(0, 3))):
            rm = r(0.5)
            if rm.any() and not any(np.array_equal(rm, x) for x, _ in D):  # (held clocks are distinct)
                D.append((rm, int(rng.integers(1, 1 << MT))))
        # the kernel's precondition: the held removes are applied to the rows
        for rm, msk in D:
            for m in range(MT):
                if (msk >> m) & 1:
                    E[m] = fg(E[m], rm)
        C = np.maximum(C0, r(0.3))
        ok = orswot_chunk_test(C0, e, oc, E, D, c2, e2, o2, E2)
        if not ok:
            continue
        n_pass += 1
        en, oc2, En, Dn = orswot_exact_step(C, e, oc.copy(), E.copy(), list(D), c2, e2, o2, E2)
        assert np.array_equal(en, e)
        if e.any():
            assert np.array_equal(oc2, oc) and np.array_equal(En, E)
            assert len(Dn) == len(D) and all(np.array_equal(a[0], b[0]) and a[1] == b[1] for a, b in zip(Dn, D))
    assert n_pass > 1000
