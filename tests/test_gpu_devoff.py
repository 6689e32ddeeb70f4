"""GPU parity: Orswot / Map lub_many with the deferred pool's CSR offsets in DEVICE memory
(crdt_orswot_lub_many_doff / crdt_map_lub_many_doff).  Results must equal the
host-offset entry points' word for word (themselves pinned against the oracle in test_gpu_orswot.py /
test_gpu_map.py) and the oracle fold per group; invalid offsets are reported on the device (Orswot
status bit 0, Map flags bit 1 of the groups they bound) and the kernels stay inside the pool."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _doff(off):
    return torch.from_numpy(np.asarray(off, dtype=np.int64)).cuda()


def _orswot_groups(G, seed, empty_every=3):
    """G groups of replicas of one shape; every `empty_every`-th group has no deferred removes."""
    parts = []
    for g in range(G):
        p = O.gen_orswot(seed * 1009 + g, 6, 40, 8, kmax=10, p_def=0.0 if g % empty_every == 0 else 0.4)
        parts.append(p)
    clock = np.stack([p[0] for p in parts])
    entries = np.stack([p[1] for p in parts])
    dcl = np.concatenate([p[3] for p in parts])
    dmem = np.concatenate([p[4] for p in parts])
    off = np.cumsum([0] + [p[3].shape[0] for p in parts]).astype(np.int64)
    return parts, clock, entries, off, dcl, dmem


@pytest.mark.parametrize("G,seed,empty_every", [(1, 1, 3), (1, 4, 100), (7, 2, 3), (300, 3, 3)])
def test_orswot_devoff_equals_host(gpu_ctx, G, seed, empty_every):
    parts, clock, entries, off, dcl, dmem = _orswot_groups(G, seed, empty_every)
    args = (to_dev(clock), to_dev(entries))
    kw = dict(def_clock=to_dev(dcl), def_members=to_dev(dmem), ctx=gpu_ctx)
    ref = cg.orswot.lub_many(*args, def_off=off, **kw)
    st = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
    got = cg.orswot.lub_many(*args, def_off=_doff(off), def_status=st, **kw)
    assert int(st.item()) == 0
    for a, b in zip(ref, got):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)
    gc, ge = to_host(got.clock), to_host(got.entries)
    for g in range(min(G, 40)):
        oc, oe, odef, _ = O.orswot_fold(*parts[g])
        np.testing.assert_array_equal(gc[g], oc)
        np.testing.assert_array_equal(ge[g], oe)
        if got.def_keep is None:
            assert odef == set()
        else:
            assert cg.orswot.deferred_set(kw["def_clock"], got.def_keep, got.def_members,
                                          int(off[g]), int(off[g + 1])) == odef


def test_orswot_devoff_no_pool(gpu_ctx):
    """def_off all zero and D = 0: no deferred output; a non-zero entry with D = 0 is reported."""
    parts, clock, entries, off, dcl, dmem = _orswot_groups(4, 9, empty_every=1)
    assert dcl.shape[0] == 0
    st = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
    got = cg.orswot.lub_many(to_dev(clock), to_dev(entries), def_off=_doff(np.zeros(5)), def_status=st,
                             ctx=gpu_ctx)
    assert int(st.item()) == 0 and got.def_keep is None
    ref = cg.orswot.lub_many(to_dev(clock), to_dev(entries), ctx=gpu_ctx)
    assert torch.equal(ref.clock, got.clock) and torch.equal(ref.entries, got.entries)
    got = cg.orswot.lub_many(to_dev(clock), to_dev(entries), def_off=_doff([0, 0, 1, 1, 1]), def_status=st,
                             ctx=gpu_ctx)
    assert int(st.item()) == 1
    assert torch.equal(ref.clock, got.clock) and torch.equal(ref.entries, got.entries)


def test_orswot_devoff_empty_members(gpu_ctx):
    """M == 0: the state is its clock — the fold is the clock lub and a deferred remove (with an
    empty member set, orswot.rs:230-250 keeps it) survives iff not dominated by the final clock.
    The status is written for every call (it was left uninitialised on this path)."""
    rng = np.random.default_rng(5)
    clock = rng.integers(0, 9, size=(3, 5, 4), dtype=np.uint64)
    dcl = rng.integers(0, 12, size=(6, 4), dtype=np.uint64)
    off = np.array([0, 2, 2, 6])
    entries = torch.empty((3, 5, 0, 4), dtype=torch.int64, device="cuda:0")
    dmem = torch.empty((6, 0), dtype=torch.int64, device="cuda:0")
    exp = clock.max(axis=1)
    keep_exp = np.array([(dcl[d] > exp[g]).any() for g in range(3) for d in range(off[g], off[g + 1])])
    for form in ("host", "device"):
        st = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
        kw = dict(def_off=_doff(off), def_status=st) if form == "device" else dict(def_off=off)
        got = cg.orswot.lub_many(to_dev(clock), entries, def_clock=to_dev(dcl), def_members=dmem, ctx=gpu_ctx, **kw)
        np.testing.assert_array_equal(to_host(got.clock), exp)
        np.testing.assert_array_equal(got.def_keep.cpu().numpy().astype(bool), keep_exp)
        if form == "device":
            assert int(st.item()) == 0
    assert keep_exp.any() and not keep_exp.all()
    st = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
    got = cg.orswot.lub_many(to_dev(clock), entries, def_off=_doff(np.zeros(4)), def_status=st, ctx=gpu_ctx)
    assert int(st.item()) == 0
    np.testing.assert_array_equal(to_host(got.clock), exp)


@pytest.mark.parametrize("bad", ["first", "last_short", "last_long", "decreasing", "past_pool"])
def test_orswot_devoff_invalid(gpu_ctx, bad):
    """Each kind of malformed offset array is reported (status bit 0 / ValueError without a status
    tensor), and the call completes with every kernel inside the pool (the clock is still exact:
    deferred removes never change it)."""
    parts, clock, entries, off, dcl, dmem = _orswot_groups(6, 5, empty_every=100)
    D = int(off[-1])
    off = off.copy()
    if bad == "first":
        off[0] = 1
    elif bad == "last_short":
        off[-1] = D - 1
    elif bad == "last_long":
        off[-1] = D + 5
    elif bad == "decreasing":
        off[2], off[3] = off[3], off[2] - 1
    else:
        off[3] = D + 1000
    kw = dict(def_clock=to_dev(dcl), def_members=to_dev(dmem), ctx=gpu_ctx)
    st = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    got = cg.orswot.lub_many(to_dev(clock), to_dev(entries), def_off=_doff(off), def_status=st, **kw)
    torch.cuda.synchronize()
    assert int(st.item()) == 1
    ref = cg.orswot.lub_many(to_dev(clock), to_dev(entries), ctx=gpu_ctx)
    assert torch.equal(ref.clock, got.clock)
    with pytest.raises(ValueError, match="def_off invalid"):
        cg.orswot.lub_many(to_dev(clock), to_dev(entries), def_off=_doff(off), **kw)


def _map_groups(G, seed, R=12, K=10, A=5):
    groups = [O.gen_map_replicas(seed * 7919 + g, R, K, A, steps=120, p_rm=0.3 if g % 4 else 0.0, p_up=0.4)
              for g in range(G)]
    V = max(O.max_vals(maps) for maps in groups)
    parts = [O.map_to_dense(maps, K, A, V) for maps in groups]
    st = {k: np.stack([p[k] for p in parts]) for k in ("clock", "ec", "vclk", "vval")}
    for k in ("def_row", "def_clock", "def_keys"):
        st[k] = np.concatenate([p[k] for p in parts])
    off = np.cumsum([0] + [p["def_row"].shape[0] for p in parts]).astype(np.int64)
    return parts, st, off


def _map_call(ctx, st, def_off, **kw):
    row = torch.from_numpy(np.asarray(st["def_row"], np.int64).astype(np.int32)).cuda()
    return cg.map.lub_many(to_dev(st["clock"]), to_dev(st["ec"]), to_dev(st["vclk"]), to_dev(st["vval"]),
                           def_off=def_off, def_row=row, def_clock=to_dev(st["def_clock"]),
                           def_keys=to_dev(st["def_keys"]), vout=16, ctx=ctx, **kw)


@pytest.mark.parametrize("mode", ["mglds=1,mrs=1", "mglds=0"])
@pytest.mark.parametrize("G,seed", [(1, 11), (5, 12), (120, 13)])
def test_map_devoff_equals_host(gpu_ctx, mode, G, seed):
    ctx = cg.Context(0)
    ctx.tune(mode)
    parts, st, off = _map_groups(G, seed)
    ref = _map_call(ctx, st, off)
    got = _map_call(ctx, st, _doff(off))
    for a, b in zip(ref, got):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)
    for g in range(min(G, 30)):
        p = parts[g]
        exp = O.map_fold(p["clock"], p["ec"], p["vclk"], p["vval"], p["def_row"], p["def_clock"], p["def_keys"], 16)
        np.testing.assert_array_equal(to_host(got.clock[g]), exp[0])
        np.testing.assert_array_equal(to_host(got.ec[g]), exp[1])
        np.testing.assert_array_equal(to_host(got.vclk[g]), exp[2])
        np.testing.assert_array_equal(to_host(got.vval[g]), exp[3])
        if got.def_keep is not None:
            assert cg.map.deferred_set(to_dev(st["def_clock"]), got.def_keep, got.def_keys,
                                       int(off[g]), int(off[g + 1])) == exp[5]


@pytest.mark.parametrize("bad", ["first", "last_short", "decreasing", "past_pool"])
def test_map_devoff_invalid(gpu_ctx, bad):
    """A malformed entry i flags bit 1 of groups i-1 and i only; the other groups stay exact."""
    parts, st, good = _map_groups(8, 21)
    G, D = 8, int(good[-1])
    off = good.copy()
    i = {"first": 0, "last_short": G, "decreasing": 4, "past_pool": 5}[bad]
    off[i] = {"first": 1, "last_short": D - 1, "decreasing": off[3] - 1, "past_pool": D + 999}[bad]
    # the rule of crdt_gpu.h, restated: entry i invalid -> groups i-1 and i flagged
    hit = set()
    for j in range(G + 1):
        v = int(off[j])
        wrong = v != 0 if j == 0 else (v != D if j == G else v > D)
        if wrong or (j > 0 and int(off[j - 1]) > v):
            hit |= {g for g in (j - 1, j) if 0 <= g < G}
    assert hit
    ref = _map_call(gpu_ctx, st, good)
    got = _map_call(gpu_ctx, st, _doff(off), check=False)
    flags = got.flags.cpu().numpy()
    for g in range(G):
        assert bool(flags[g] & 2) == (g in hit), (g, flags.tolist())
        if g not in hit:  # both bounding entries valid: the group's fold is exact
            assert torch.equal(ref.ec[g], got.ec[g]) and torch.equal(ref.vval[g], got.vval[g]), g
    with pytest.raises(ValueError, match="device def_off"):
        _map_call(gpu_ctx, st, _doff(off))
