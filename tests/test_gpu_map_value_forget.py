"""GPU: Causal::forget of whole value-typed Map states (round 5; crdt_map_counter_forget_batch,
crdt_map_orswot_forget_batch) against the oracle's Map.forget (map.rs:85-114 with gcounter.rs:51-53,
pncounter.rs:78-81, orswot.rs:150-183) on op-replay states with deferred removes at every level."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _forget_clocks(rng, clock, mode):
    """Per-state forget clocks: below the state's clock (partial forgets), its clock itself (every
    dot forgotten) or zero (nothing)."""
    c = clock.astype(np.int64)
    if mode == "below":
        return (rng.integers(0, c + 1) * (rng.random(c.shape) < 0.7)).astype(np.uint64)
    if mode == "all":
        return clock.copy()
    return np.zeros_like(clock)


@pytest.mark.parametrize("W", [1, 2])
@pytest.mark.parametrize("mode", ["below", "all", "zero"])
def test_map_counter_forget(gpu_ctx, W, mode):
    N, K, A = 24, 5, 6
    maps = O.map_counter_objects(N, K, A, W, seed=40, steps=220)  # (a seed whose replicas hold removes)
    d = O.map_counter_to_dense(maps, K, A, W)
    rng = np.random.default_rng(W * 7 + len(mode))
    y = _forget_clocks(rng, d["clock"], mode)
    clock, ec, val = to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["val"])
    D = d["def_row"].shape[0]
    dcl = to_dev(d["def_clock"]) if D else None
    dst = torch.from_numpy(np.asarray(d["def_row"], np.int64).astype(np.int32)).cuda() if D else None
    keep = cg.map.counter_forget_batch(clock, ec, val, to_dev(y), def_clock=dcl, def_state=dst, ctx=gpu_ctx)
    c, e, v = to_host(clock), to_host(ec), to_host(val)
    kp = keep.cpu().numpy() if keep is not None else np.zeros(0, np.uint8)
    hd = to_host(dcl) if D else np.zeros((0, A), np.uint64)
    assert D > 0
    for n in range(N):
        exp = maps[n].copy()
        exp.forget(O.VClock({a: int(x) for a, x in enumerate(y[n]) if x}))
        dfr = [(hd[j], O.bitmap_members(d["def_keys"][j])) for j in np.flatnonzero(d["def_row"] == n) if kp[j]]
        got = O.dense_to_map_counter(c[n], e[n], v[n], dfr)
        assert got == exp, n


def _orswot_states(ctx, maps, K, M, A):
    """Each replica folded alone (G = N groups of R = 1): the states in the lub_many output layout."""
    N = len(maps)
    d = O.map_orswot_to_dense(maps, K, M, A)
    D = d["def_row"].shape[0]
    off = [0]
    for m in maps:
        off.append(off[-1] + len(m.deferred))
    kw = dict(def_off=off, def_row=torch.zeros(D, dtype=torch.int32, device="cuda:0"),
              def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"])) if D else {}
    Dv = int(d["vd_off"][-1])
    vkw = dict(vd_clock=to_dev(d["vd_clock"]), vd_mem=to_dev(d["vd_members"])) if Dv else {}
    shp = lambda x: to_dev(x.reshape((N, 1) + x.shape[1:]))  # noqa: E731
    res = cg.map.orswot_lub_many(shp(d["clock"]), shp(d["ec"]), shp(d["oc"]), shp(d["ent"]), to_dev(d["vd_off"]),
                                 ctx=ctx, **vkw, **kw)
    return res, kw, off


def _decode_orswot(res, kw, off, n, keep2):
    c, e, o, m = to_host(res.clock), to_host(res.ec), to_host(res.oc), to_host(res.ent)
    vn = res.vd_n.cpu().numpy()
    vc, vm = to_host(res.vd_clock), to_host(res.vd_mem)
    mw = (lambda k, i: vm[n, k, i]) if vm.ndim == 4 else (lambda k, i: vm[n, k, i:i + 1])  # noqa: E731
    vd = {k: [(vc[n, k, i], O.bitmap_members(mw(k, i))) for i in range(int(vn[n, k]))] for k in range(e.shape[1])}
    dfr = []
    if kw:
        keep1 = res.def_keep.cpu().numpy()
        dcl, dk = to_host(kw["def_clock"]), to_host(res.def_keys)
        dfr = [(dcl[j], O.bitmap_members(dk[j])) for j in range(off[n], off[n + 1]) if keep1[j] and keep2[j]]
    return O.dense_to_map_orswot(c[n], e[n], o[n], m[n], vd, dfr)


@pytest.mark.parametrize("M,A,mode", [(4, 5, "below"), (6, 4, "all"), (3, 6, "zero"), (70, 8, "below"),
                                      (5, 80, "below")])
def test_map_orswot_forget(gpu_ctx, M, A, mode):
    N, K = 20, 4
    maps = O.map_orswot_objects(N, K, M, A, seed=50 + M + A, steps=200, p_vrm=0.45)
    res, kw, off = _orswot_states(gpu_ctx, maps, K, M, A)
    rng = np.random.default_rng(M * 3 + A)
    y = _forget_clocks(rng, to_host(res.clock), mode)
    D = off[-1]
    dcl = kw["def_clock"].clone() if D else None
    dst = torch.tensor([n for n in range(N) for _ in range(off[n + 1] - off[n])], dtype=torch.int32,
                       device="cuda:0") if D else None
    exps = [O.map_fold_objects([m]) for m in maps]
    if any(len(e.val.deferred) > cg.map.VD_CAP for x in exps for e in x.entries.values()):
        pytest.skip("nested deferred past the kernel's capacity")
    keep2 = cg.map.orswot_forget_batch(res, to_dev(y), def_clock=dcl, def_state=dst, ctx=gpu_ctx)
    kw2 = dict(kw, def_clock=dcl) if D else kw
    k2 = keep2.cpu().numpy() if keep2 is not None else None
    nested = 0
    for n in range(N):
        exp = exps[n]
        exp.forget(O.VClock({a: int(x) for a, x in enumerate(y[n]) if x}))
        nested += sum(len(e.val.deferred) for e in exp.entries.values())
        got = _decode_orswot(res, kw2, off, n, k2)
        assert got.clock == exp.clock, n
        assert got.entries == exp.entries, n
        assert got.deferred == exp.deferred, n
    if mode == "below":
        assert nested > 0
