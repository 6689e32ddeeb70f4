"""GPU parity at shapes past the fast kernels' register limits (VERDICT r3 missing #2): the
reference's VClock / MVReg / Map are unbounded in actors and values (vclock.rs:56-60,
mvreg.rs:33-35, map.rs:31-38), so the batched forms must be too.  crdt_map_lub_many runs the
workgroup-per-key fold (csrc/map_wide.hip) for A > 256 or V > 8; its results must equal the oracle's
restated left fold (oracle/ref_fold.cpp oracle_map_fold) word for word, deferred removes included."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host
from test_gpu_map import _chain_dense, _random_dense

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402


def _map_gpu(ctx, d, vout):
    D = d["def_clock"].shape[0]
    kw = {}
    if D:
        kw = dict(def_off=[0, D], def_row=torch.from_numpy(np.asarray(d["def_row"], np.int64).astype(np.int32)).cuda(),
                  def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"]))
    res = cg.map.lub_many(to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["vclk"]), to_dev(d["vval"]), vout=vout,
                          ctx=ctx, **kw)
    return res, kw


def _map_check(ctx, d):
    peak = np.zeros(d["ec"].shape[1], np.uint64)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"], 64,
                     peak=peak)
    vout = max(1, int(exp[4].max()) if exp[4].size else 1)
    if int(peak.max()) > 16:  # beyond the state capacity: reported, never wrong
        with pytest.raises(cg.map.MapCapacityError):
            _map_gpu(ctx, d, vout)
        return None
    res, kw = _map_gpu(ctx, d, vout)
    np.testing.assert_array_equal(to_host(res.clock), exp[0])
    np.testing.assert_array_equal(to_host(res.ec), exp[1])
    np.testing.assert_array_equal(to_host(res.vclk), exp[2])
    np.testing.assert_array_equal(to_host(res.vval), exp[3])
    np.testing.assert_array_equal(res.nval.cpu().numpy(), exp[4])
    got = cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys) if kw else set()
    assert got == exp[5]
    return exp


@pytest.mark.parametrize("seed,R,K,A,V,cmax,nchain", [
    (1, 40, 5, 300, 2, 6, 3), (2, 25, 4, 1024, 2, 5, 3), (3, 12, 3, 257, 1, 4, 3), (4, 60, 6, 300, 3, 4, 3),
    (5, 30, 4, 64, 12, 5, 12), (6, 20, 3, 300, 12, 4, 12), (7, 3, 2, 1024, 9, 3, 9), (8, 90, 70, 300, 2, 3, 3),
])
def test_map_lub_many_wide(gpu_ctx, seed, R, K, A, V, cmax, nchain):
    """Dense states at A = 257 .. 1,024 actors and V = 9 / 12 value slots, with deferred removes
    (value clocks on `nchain` actors per key, so folds keep up to nchain concurrent values): the
    wide fold equals the reference left fold, every case run (none needs more than 16 values)."""
    rng = np.random.default_rng(seed)
    d = _chain_dense(rng, R, K, A, V, cmax, nchain=nchain)
    assert _map_check(gpu_ctx, d) is not None


@pytest.mark.parametrize("seed,R,K,A,V,cmax", [(11, 40, 5, 300, 2, 6), (12, 20, 3, 300, 12, 4)])
def test_map_lub_many_wide_arbitrary(gpu_ctx, seed, R, K, A, V, cmax):
    """Arbitrary states: a fold needing more than 16 values is reported (MapCapacityError), any other
    equals the reference fold."""
    rng = np.random.default_rng(seed)
    _map_check(gpu_ctx, _random_dense(rng, R, K, A, V, cmax))


@pytest.mark.parametrize("R,V,A", [(1, 12, 40), (2, 6, 300), (1, 16, 1024), (3, 12, 300)])
def test_map_wide_many_concurrent_values(gpu_ctx, R, V, A):
    """Registers holding V concurrent values (every write by its own actor): the fold keeps all
    R * V of them (up to the 16-value state), in Vec order."""
    K = 3
    clock = np.zeros((R, A), np.uint64)
    ec = np.zeros((R, K, A), np.uint64)
    vclk = np.zeros((R, K, V, A), np.uint64)
    vval = np.zeros((R, K, V), np.uint64)
    for r in range(R):
        for t in range(V):
            a = (r * V + t) * 7 % A
            clock[r, a] = 1
            ec[r, :, a] = 1
            vclk[r, :, t, a] = 1
            vval[r, :, t] = 100 * r + t
    d = dict(clock=clock, ec=ec, vclk=vclk, vval=vval, def_row=np.zeros(0, np.uint64),
             def_clock=np.zeros((0, A), np.uint64), def_keys=np.zeros((0, 1), np.uint64))
    exp = _map_check(gpu_ctx, d)
    assert exp is None or int(exp[4].max()) == R * V


def test_map_wide_op_replay(gpu_ctx):
    """States built by the reference's own op semantics (oracle op replay: writes with read
    contexts, removes, out-of-order delivery leaving deferred removes) with 300 actor slots."""
    maps = O.gen_map_replicas(84, 40, 10, 6, steps=300, p_rm=0.3, p_up=0.4)
    V = max(1, O.max_vals(maps))
    d = O.map_to_dense(maps, 10, 6, V)
    A = 300  # the 6 live actors spread over 300 dense columns (actors interned sparsely)
    cols = np.array([0, 37, 111, 150, 233, 299])

    def widen(x):
        out = np.zeros(x.shape[:-1] + (A,), np.uint64)
        out[..., cols] = x
        return out

    wd = dict(clock=widen(d["clock"]), ec=widen(d["ec"]), vclk=widen(d["vclk"]), vval=d["vval"], def_row=d["def_row"],
              def_clock=widen(d["def_clock"]), def_keys=d["def_keys"])
    exp = _map_check(gpu_ctx, wd)
    assert exp is not None and exp[5]  # surviving deferred removes exercised
