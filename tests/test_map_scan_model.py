"""Soundness of the Map fold kernel's speculative no-op scan (rust-crdt_amd/csrc/map.hip,
map_noop_steps): a numpy model of its per-step test, run beside the dense restatement of the
reference fold (oracle.dense_map_fold, map.rs:140-220).  Whenever the test declares a step a
no-op, the exact entry join of that step must leave (present, entry clock, MVReg values in Vec
order) unchanged.  The model uses the exact acc clock; the kernel uses a possibly older one,
which only makes its test stricter (every Cs condition is monotone)."""
import numpy as np
import pytest

import oracle as O

z = np.uint64(0)


def _vals_key(vals):
    return [(tuple(int(x) for x in c), int(v)) for c, v in vals]


def _noop_test(present, e, vals, e2, v2, Cs, Co):
    """The kernel's scan test for one step (None: the scan does not run, own values not an
    antichain)."""
    p2 = bool(e2.any())
    if not present:
        return (not p2) or bool(np.all(e2 <= Cs))
    if any(O._lt(c, c2) for c, _ in vals for c2, _ in vals):
        return None
    if not p2:
        ri = np.where(Co > e, Co, z)
        return bool(np.all((e == 0) | (e > Co))) and all(np.all((c == 0) | (c > ri)) for c, _ in vals)
    if not (np.all((e2 <= e) | (e2 <= Cs)) and np.all((e == 0) | (e == e2) | (e > Co))):
        return False
    dl = np.where(e2 > e, e2, z)
    if not all(np.all((c == 0) | (c > dl)) for c, _ in vals):
        return False
    for t, _ in v2:
        if not (any(np.all(t <= c) for c, _ in vals) or np.all(t <= dl)):
            return False
    return True


U64MAX = np.uint64(0xFFFFFFFFFFFFFFFF)


def _noop_test_thr(present, e, vals, e2, v2, Cs, Co):
    """map_noop_steps3's form of the same test: per-actor thresholds TB = max(e, min(Cs, m1)) and
    TO = e > 0 ? e - 1 : m1, m1 = (min of the nonzero own value clocks) - 1 or UINT64_MAX."""
    p2 = bool(e2.any())
    m1 = np.full(e.shape, U64MAX)
    for c, _ in vals:
        m1 = np.minimum(m1, np.where(c != 0, c - np.uint64(1), U64MAX))
    TB = np.maximum(e, np.minimum(Cs, m1))
    if not present:
        return (not p2) or bool(np.all(e2 <= TB))
    if any(O._lt(c, c2) for c, _ in vals for c2, _ in vals):
        return None
    with np.errstate(over="ignore"):
        TO = np.where(e > 0, e - np.uint64(1), m1)
        em1 = e - np.uint64(1)  # wraps to UINT64_MAX at e == 0
    if not p2:
        return bool(np.all(Co <= TO))
    if not np.all((e2 <= TB) & ((em1 >= Co) | (e == e2))):
        return False
    dl = np.where(e2 > e, e2, z)
    for t, _ in v2:
        if not (any(np.all(t <= c) for c, _ in vals) or np.all(t <= dl)):
            return False
    return True


def _join(present, e, vals, e2, v2, Cs, Co, A):
    """The entry join of one step (oracle.dense_map_fold steps 1, map.rs:142-210)."""
    p2 = bool(e2.any())
    if present and not p2:
        if np.all(Co >= e):
            return False, np.zeros(A, np.uint64), []
        e = np.where(e > Co, e, z).astype(np.uint64)
        return True, e, O._forget_vals(vals, np.where(Co > e, Co, z))
    if p2 and not present:
        if not np.all(Cs >= e2):
            e = np.where(e2 > Cs, e2, z).astype(np.uint64)
            return True, e, O._forget_vals(v2, np.where(Cs > e, Cs, z))
        return present, e, vals
    if present and p2:
        common = np.maximum(np.where(e == e2, e, z), np.maximum(np.where(e2 > Cs, e2, z), np.where(e > Co, e, z)))
        if not common.any():
            return False, np.zeros(A, np.uint64), []
        vals = O._mv_merge(vals, v2)
        dl = np.maximum(e, e2)
        return True, common.astype(np.uint64), O._forget_vals(vals, np.where(dl > common, dl, z))
    return present, e, vals


def _check_fold(d):
    clock, ec, vclk, vval = d["clock"], d["ec"], d["vclk"], d["vval"]
    R, K, A = ec.shape
    V = vclk.shape[2]
    t, P = O.map_drop_steps(clock, d["def_row"], d["def_clock"])
    rows = np.asarray(d["def_row"], np.int64)
    n_noop = 0
    for k in range(K):
        kb = [x for x in range(len(rows)) if (int(d["def_keys"][x][k // 64]) >> (k % 64)) & 1]
        present, e, vals = False, np.zeros(A, np.uint64), []
        for i in range(R):
            Cs, Co = P[i], clock[i]
            e2 = ec[i, k]
            v2 = [(vclk[i, k, s].copy(), int(vval[i, k, s])) for s in range(V) if vclk[i, k, s].any()]
            verdict = _noop_test(present, e, vals, e2, v2, Cs, Co)
            assert _noop_test_thr(present, e, vals, e2, v2, Cs, Co) == verdict, f"key {k} step {i}: threshold form differs"
            np_, ne, nv = _join(present, e, vals, e2, v2, Cs, Co, A)
            if verdict:
                n_noop += 1
                assert np_ == present and np.array_equal(ne, e) and _vals_key(nv) == _vals_key(vals), \
                    f"key {k} step {i}: declared a no-op but the join changes the state"
            present, e, vals = np_, ne, nv
            act = [x for x in kb if rows[x] <= i <= t[x]]
            if act and present:
                ceil = np.max(np.stack([d["def_clock"][x] for x in act]), axis=0)
                e = np.where(e > ceil, e, z).astype(np.uint64)
                if not e.any():
                    present, vals = False, []
                else:
                    vals = O._forget_vals(vals, ceil)
    return n_noop


@pytest.mark.parametrize("seed", range(40))
def test_scan_sound_op_replay(seed):
    rng = np.random.default_rng(seed)
    K, A = int(rng.integers(1, 20)), int(rng.integers(1, 9))
    R = int(rng.integers(2, 40))
    p_rm = float(rng.choice([0.15, 0.3, 0.45]))
    maps = O.gen_map_replicas(seed, R, K, A, steps=int(rng.integers(20, 300)), p_rm=p_rm, p_up=0.7 - p_rm)
    d = O.map_to_dense(maps, K, A, O.max_vals(maps))
    _check_fold(d)


@pytest.mark.parametrize("seed", range(40))
def test_scan_sound_arbitrary(seed):
    rng = np.random.default_rng(1000 + seed)
    R, K, A, V = int(rng.integers(2, 30)), int(rng.integers(1, 6)), int(rng.integers(1, 6)), int(rng.integers(1, 3))
    cmax = int(rng.choice([2, 3, 5]))
    clock = rng.integers(0, cmax, size=(R, A)).astype(np.uint64)
    ec = rng.integers(0, cmax, size=(R, K, A)).astype(np.uint64)
    ec[rng.random((R, K)) < 0.3] = 0
    vclk = rng.integers(0, cmax, size=(R, K, V, A)).astype(np.uint64)
    vval = rng.integers(0, 5, size=(R, K, V)).astype(np.uint64)
    D = int(rng.integers(0, R // 2 + 1))
    def_row = np.sort(rng.integers(0, R, size=D)).astype(np.uint64)
    def_clock = rng.integers(0, cmax + 1, size=(D, A)).astype(np.uint64)
    def_keys = rng.integers(0, 2 ** 63, size=(D, 1)).astype(np.uint64)
    _check_fold(dict(clock=clock, ec=ec, vclk=vclk, vval=vval, def_row=def_row, def_clock=def_clock,
                     def_keys=def_keys))


def test_scan_sound_synthetic():
    """The config-4 generator's replicas (sampled keys): most steps are no-ops."""
    seed, R, K, A, kmax = 5, 400, 24, 8, 40
    dfr = O.synth_map_deferred(seed, R, K, A, kmax, p_def=0.2)
    d = O.synth_map(seed, R, K, A, 2, kmax, deferred=dfr)
    d.update(def_row=dfr[0], def_clock=dfr[1], def_keys=dfr[2])
    n = _check_fold(d)
    assert n > R * K // 2


@pytest.mark.parametrize("seed", range(20))
def test_threshold_form_edges(seed):
    """The threshold form on counters at 0, 1 and UINT64_MAX (the wrap cases of e - 1 and m1)."""
    rng = np.random.default_rng(7000 + seed)
    pool = np.array([0, 1, 2, 3, 0xFFFFFFFFFFFFFFFE, 0xFFFFFFFFFFFFFFFF], np.uint64)
    for _ in range(300):
        A = int(rng.integers(1, 5))
        pick = lambda: pool[rng.integers(0, len(pool), size=A)]  # noqa: E731
        e, e2, Cs, Co = pick(), pick(), pick(), pick()
        if rng.random() < 0.3:
            e2[:] = 0
        present = bool(e.any())
        nv = int(rng.integers(0, 3)) if present else 0
        vals = [(pick(), 0) for _ in range(nv)]
        v2 = [(pick(), 0) for _ in range(int(rng.integers(0, 3)))] if e2.any() else []
        assert _noop_test_thr(present, e, vals, e2, v2, Cs, Co) == _noop_test(present, e, vals, e2, v2, Cs, Co)


def test_chunk_clock_max_form_is_sound_but_weaker():
    """Design probe: testing a 16-replica chunk with its clock max in place of each
    step's replica clock would let the staged chunk drop its replica-clock quarter.  The max form is
    sound (a larger Co only fails more of the Co-tests) but skips far fewer chunks on the config-4
    generator (98.7% -> 85.7% at 4,096 replicas x 6 keys), so the RS path keeps per-step clocks."""
    R, K, A, V, kmax, C = 512, 4, 32, 2, 256, 16
    d = O.synth_map(5, R, K, A, V, kmax)
    clock, ec, vclk, vval = d["clock"], d["ec"], d["vclk"], d["vval"]
    P = np.zeros((R + 1, A), np.uint64)
    for i in range(R):
        P[i + 1] = np.maximum(P[i], clock[i])
    n = sk_co = sk_cm = 0
    for k in range(K):
        present, e, vals = False, np.zeros(A, np.uint64), []
        for c0 in range(0, R, C):
            cm = clock[c0:c0 + C].max(axis=0)
            ok_co = ok_cm = True
            for i in range(c0, min(c0 + C, R)):
                v2 = [(vclk[i, k, s].copy(), int(vval[i, k, s])) for s in range(V) if vclk[i, k, s].any()]
                a = _noop_test_thr(present, e, vals, ec[i, k], v2, P[c0], clock[i])
                b = _noop_test_thr(present, e, vals, ec[i, k], v2, P[c0], cm)
                assert not b or a, (k, i)  # the max form never skips a step the exact form keeps
                ok_co &= bool(a)
                ok_cm &= bool(b)
            n += 1
            sk_co += ok_co
            sk_cm += ok_cm
            for i in range(c0, min(c0 + C, R)):
                v2 = [(vclk[i, k, s].copy(), int(vval[i, k, s])) for s in range(V) if vclk[i, k, s].any()]
                present, e, vals = _join(present, e, vals, ec[i, k], v2, P[i], clock[i], A)
    assert sk_cm <= sk_co and sk_co > 0.9 * n
