"""Shared by the Orswot batched-apply tests (CPU dense restatement and GPU kernel): dense
<-> oracle object conversion and op-stream generators."""
import numpy as np

import oracle as O


def dense_states(states, M, A, Dcap):
    N = len(states)
    Mw = (M + 63) // 64
    clock = np.zeros((N, A), np.uint64)
    entries = np.zeros((N, M, A), np.uint64)
    dcl = np.zeros((N, Dcap, A), np.uint64)
    dmb = np.zeros((N, Dcap, Mw), np.uint64)
    cnt = np.zeros(N, np.int32)
    for s, o in enumerate(states):
        for a, v in o.clock.dots.items():
            clock[s, a] = v
        for m, c in o.entries.items():
            for a, v in c.dots.items():
                entries[s, m, a] = v
        for d, (k, ms) in enumerate(o.deferred.items()):
            for a, v in k.dots.items():
                dcl[s, d, a] = v
            for m in ms:
                dmb[s, d, m // 64] |= np.uint64(1) << np.uint64(m % 64)
        cnt[s] = len(o.deferred)
    return clock, entries, dcl, dmb, cnt


def op_tuple(op):
    if isinstance(op, O.OrswotAdd):
        return ("add", op.dot.actor, op.dot.counter, sorted(op.members))
    return ("rm", dict(op.clock.dots), sorted(op.members))


def to_object(clock, entries, dcl, dmb, cnt, s):
    o = O.Orswot()
    o.clock = O.VClock({a: int(v) for a, v in enumerate(clock[s]) if v})
    for m in range(entries.shape[1]):
        if entries[s, m].any():
            o.entries[m] = O.VClock({a: int(v) for a, v in enumerate(entries[s, m]) if v})
    for d in range(int(cnt[s])):
        k = O.VClock({a: int(v) for a, v in enumerate(dcl[s, d]) if v})
        assert k not in o.deferred, "deferred clocks must stay pairwise distinct"
        o.deferred[k] = set(O.bitmap_members(dmb[s, d]))
    return o


def oracle_streams(states, streams):
    out = []
    for o, ops in zip(states, streams):
        o = o.copy()
        for op in ops:
            o.apply(op)
        out.append(o)
    return out


def map_orswot(v, fa, fm):
    o = O.Orswot()
    o.clock = O.VClock({fa(a): c for a, c in v.clock.dots.items()})
    o.entries = {fm(m): O.VClock({fa(a): c for a, c in e.dots.items()}) for m, e in v.entries.items()}
    o.deferred = {O.VClock({fa(a): c for a, c in k.dots.items()}): {fm(m) for m in ms} for k, ms in v.deferred.items()}
    return o


def replay_streams(seed, n_states, n_origins, M, n_ops):
    rng = np.random.default_rng(seed)
    origins = [O.Orswot() for _ in range(n_origins)]
    ops = []
    for _ in range(n_ops):
        a = int(rng.integers(0, n_origins))
        o = origins[a]
        r = rng.random()
        if r < 0.08:  # origins gossip, so remove contexts carry other actors' dots
            o.merge(origins[int(rng.integers(0, n_origins))])
            continue
        m = int(rng.integers(0, M))
        if r < 0.65 or not o.entries:
            ms = [m] if rng.random() < 0.8 else list(rng.choice(M, size=min(M, 3), replace=False))
            op = O.OrswotAdd(o.read().derive_add_ctx(a).dot, ms)
        else:
            m = list(o.entries)[int(rng.integers(0, len(o.entries)))] if rng.random() < 0.7 else m
            op = O.OrswotRm(o.contains(m).derive_rm_ctx().clock, [m])
        o.apply(op)
        ops.append(op)
    streams = []
    for _ in range(n_states):
        keep = rng.random(len(ops)) < rng.uniform(0.4, 1.0)
        idx = np.flatnonzero(keep)
        # mostly causal order with local swaps (out-of-order delivery)
        idx = idx[np.argsort(idx + rng.normal(0, rng.uniform(0, 12), size=idx.shape[0]))]
        idx = idx[:int(rng.integers(len(idx) // 2, len(idx) + 1))]  # cut: late removes stay deferred
        streams.append([ops[i] for i in idx])
    return streams


def random_ops(rng, n, M, A, kmax):
    ops = []
    for _ in range(n):
        ms = [int(x) for x in rng.choice(M, size=int(rng.integers(0, min(M, 4) + 1)), replace=True)]
        if rng.random() < 0.6:
            ops.append(O.OrswotAdd(O.Dot(int(rng.integers(0, A)), int(rng.integers(0, kmax + 4))), ms))
        else:
            rm = rng.integers(0, kmax + 4, size=A) * (rng.random(A) < 0.5)
            ops.append(O.OrswotRm(O.VClock({a: int(v) for a, v in enumerate(rm) if v}), ms))
    return ops


def arbitrary_case(seed, N, M, A, max_ops=40):
    """Arbitrary well-formed-ish states (gen_orswot replicas with deferred removes) and random
    ops: any actor / counter / rm clock, duplicate members, empty member lists and clocks."""
    rng = np.random.default_rng(seed)
    clock, entries, off, dcl, dmem = O.gen_orswot(seed, N, M, A, kmax=8, p_def=0.5)
    states = []
    for s in range(N):
        o = O.Orswot()
        o.clock = O.VClock({a: int(v) for a, v in enumerate(clock[s]) if v})
        for m in range(M):
            if entries[s, m].any():
                o.entries[m] = O.VClock({a: int(v) for a, v in enumerate(entries[s, m]) if v})
        for d in range(int(off[s]), int(off[s + 1])):
            k = O.VClock({a: int(v) for a, v in enumerate(dcl[d]) if v})
            o.deferred.setdefault(k, set()).update(O.bitmap_members(dmem[d]))
        states.append(o)
    streams = [random_ops(rng, int(rng.integers(0, max_ops)), M, A, 8) for _ in range(N)]
    return states, streams
