"""GPU parity: batched Causal::forget of whole Orswot (orswot.rs:150-183) and Map<K, MVReg>
(map.rs:85-114, mvreg.rs:88-104) states vs the oracle objects' forget, one clock per state or
one shared clock.  When two surviving deferred rm clocks of a state collide after the forget,
the reference keeps one of them by HashMap iteration order (unspecified): there the test
checks the kept clocks and that the oracle's surviving entry is one of the kernel's rows."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host
from orswot_apply_util import arbitrary_case

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _check_deferred(rows, oracle_deferred, A):
    """rows: [(rm tuple, frozenset)] kept by the kernel for one state."""
    clocks = [r for r, _ in rows]
    exp = {(tuple(k.get(a) for a in range(A)), frozenset(ms)) for k, ms in oracle_deferred.items()}
    if len(set(clocks)) == len(clocks):
        assert set(rows) == exp
    else:  # collision: unspecified which member set the reference keeps
        assert set(clocks) == {c for c, _ in exp}
        assert exp <= set(rows)


@pytest.mark.parametrize("seed,N,M,A,shared", [(1, 40, 16, 8, False), (2, 30, 70, 64, True),
                                               (3, 12, 130, 33, False), (4, 50, 5, 2, False)])
def test_orswot_forget_batch(gpu_ctx, seed, N, M, A, shared):
    states, _ = arbitrary_case(seed, N, M, A, max_ops=1)
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 10, size=(1 if shared else N, A)).astype(np.uint64) * (rng.random((1 if shared else N, A)) < 0.7)
    y = y.astype(np.uint64)
    clock = np.zeros((N, A), np.uint64)
    entries = np.zeros((N, M, A), np.uint64)
    dcl, dmem, dstate = [], [], []
    Mw = (M + 63) // 64
    for s, o in enumerate(states):
        for a, v in o.clock.dots.items():
            clock[s, a] = v
        for m, c in o.entries.items():
            for a, v in c.dots.items():
                entries[s, m, a] = v
        for k, ms in o.deferred.items():
            row = np.zeros(A, np.uint64)
            for a, v in k.dots.items():
                row[a] = v
            bits = np.zeros(Mw, np.uint64)
            for m in ms:
                bits[m // 64] |= np.uint64(1) << np.uint64(m % 64)
            dcl.append(row)
            dmem.append(bits)
            dstate.append(s)
    tc, te = to_dev(clock), to_dev(entries)
    ty = to_dev(y[0] if shared else y)
    tdc = to_dev(np.array(dcl, np.uint64).reshape(-1, A))
    tds = torch.tensor(dstate, dtype=torch.int32, device="cuda:0")
    keep = cg.orswot.forget_batch(tc, te, ty, tdc, tds, ctx=gpu_ctx)
    c, e, dc = to_host(tc), to_host(te), to_host(tdc)
    kp = keep.cpu().numpy() if keep is not None else np.zeros(0, np.uint8)
    for s, o in enumerate(states):
        o = o.copy()
        o.forget(O.VClock({a: int(v) for a, v in enumerate(y[0 if shared else s]) if v}))
        assert c[s].tolist() == [o.clock.get(a) for a in range(A)], s
        for m in range(M):
            exp = o.entries.get(m)
            assert e[s, m].tolist() == ([exp.get(a) for a in range(A)] if exp else [0] * A), (s, m)
        rows = [(tuple(int(v) for v in dc[d]), frozenset(O.bitmap_members(dmem[d])))
                for d in range(len(dstate)) if dstate[d] == s and kp[d]]
        _check_deferred(rows, o.deferred, A)


# even A <= 128 runs map_forget_vec2_kernel (16-byte pieces), odd A <= 64 the narrow kernel, A = 65
# (odd, > 64) the wide one; mfv2=0 forces the narrow kernel for an even A
@pytest.mark.parametrize("seed,R,K,A,shared,tune", [
    (5, 24, 16, 8, False, ""), (6, 16, 40, 32, True, ""), (7, 10, 8, 65, False, ""), (8, 12, 20, 100, False, ""),
    (9, 20, 12, 7, True, ""), (10, 16, 24, 32, False, "mfv2=0")])
def test_map_forget_batch(gpu_ctx, seed, R, K, A, shared, tune):
    if tune:
        gpu_ctx = cg.Context(0)
        gpu_ctx.tune(tune)
    maps = O.gen_map_replicas(seed, R, K, A, steps=150)
    V = max(1, O.max_vals(maps))
    d = O.map_to_dense(maps, K, A, V)
    rng = np.random.default_rng(seed)
    y = (rng.integers(0, 12, size=(1 if shared else R, A)) * (rng.random((1 if shared else R, A)) < 0.6)).astype(np.uint64)
    tc, tec, tvc, tvv = (to_dev(d[k]) for k in ("clock", "ec", "vclk", "vval"))
    D = d["def_clock"].shape[0]
    kw = {}
    if D:
        kw = dict(def_clock=to_dev(d["def_clock"]),
                  def_state=torch.from_numpy(d["def_row"].astype(np.int32)).cuda())
    keep = cg.map.forget_batch(tc, tec, tvc, tvv, to_dev(y[0] if shared else y), ctx=gpu_ctx, **kw)
    c, ec, vc, vv = to_host(tc), to_host(tec), to_host(tvc), to_host(tvv)
    kp = keep.cpu().numpy() if keep is not None else np.zeros(0, np.uint8)
    dc = to_host(kw["def_clock"]) if D else np.zeros((0, A), np.uint64)
    for r, m in enumerate(maps):
        m = m.copy()
        m.forget(O.VClock({a: int(v) for a, v in enumerate(y[0 if shared else r]) if v}))
        got = O.dense_to_map(c[r], ec[r], vc[r], vv[r])
        assert got.clock == m.clock and got.entries == m.entries, r
        # emptied value slots carry value 0; dropped keys have all-zero slots
        assert not vc[r][~ec[r].any(axis=1)].any()
        assert not vv[r][~vc[r].any(axis=2)].any()
        rows = [(tuple(int(v) for v in dc[i]), frozenset(O.bitmap_members(d["def_keys"][i])))
                for i in range(D) if int(d["def_row"][i]) == r and kp[i]]
        _check_deferred(rows, m.deferred, A)
