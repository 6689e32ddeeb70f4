"""The sharded entry points on one GPU without a process group (world = 1) must equal the
plain lub: they run the real kernels end to end (the N>1 exchange is covered by the gloo
tests in test_dist_cpu.py and by bench.py --gpus N)."""
import numpy as np
import pytest
import torch

import oracle as O
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import dist as cdist  # noqa: E402


def test_counters_sharded_world1(gpu_ctx):
    x = to_dev(O.synth_matrix(5, 3000, 100, 0))
    out = cdist.lub_many_sharded("gcounter", x)
    assert torch.equal(out, cg.gcounter.lub_many(x))
    g = to_dev(O.synth_matrix(6, 300, 9, 1))
    assert torch.equal(cdist.lub_many_sharded("gset", g), cg.gset.lub_many(g))


def test_lww_sharded_world1(gpu_ctx):
    m = to_dev(O.synth_matrix(8, 2, 500, 2) % np.uint64(5))
    v = to_dev(O.synth_matrix(8, 2, 500, 3) % np.uint64(2))
    fm, fv, fc = cdist.lwwreg_lub_many_sharded(m, v, base=0)
    res = cg.lwwreg.lub_many(m, v)
    assert torch.equal(fm, res.marker) and torch.equal(fv, res.val) and torch.equal(fc, res.first_conflict)


def test_orswot_sharded_world1(gpu_ctx):
    clock, entries, off, dcl, dmem = O.gen_orswot(12, 20, 50, 8, kmax=10)
    D = dcl.shape[0]
    res = cdist.orswot_lub_many_sharded(to_dev(clock)[None], to_dev(entries)[None], to_dev(dcl),
                                        to_dev(dmem), torch.zeros(D, dtype=torch.int64, device="cuda"))
    oc, oe, odef, _ = O.orswot_fold(clock, entries, off, dcl, dmem)
    np.testing.assert_array_equal(to_host(res.clock)[0], oc)
    np.testing.assert_array_equal(to_host(res.entries)[0], oe)
    assert cg.orswot.deferred_set(to_dev(dcl), res.def_keep, res.def_members) == odef


def test_map_key_shards_world1(gpu_ctx):
    """Each key range folded on its own (the per-rank work of map_lub_many_sharded) equals the
    oracle's whole fold restricted to it; the expanded remove key sets union to the oracle's."""
    maps = O.gen_map_replicas(31, 40, 37, 6, steps=300, p_rm=0.3, p_up=0.4)
    d = O.map_to_dense(maps, 37, 6, O.max_vals(maps))
    D = d["def_row"].shape[0]
    assert D > 0
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"], 8)
    kw = dict(def_off=[0, D], def_row=torch.from_numpy(d["def_row"].astype(np.int32)).cuda(),
              def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"]))
    union = None
    for k0, k1 in [(0, 13), (13, 20), (20, 37)]:
        res = cdist.map_lub_many_sharded(to_dev(d["clock"])[None], to_dev(d["ec"][:, k0:k1])[None],
                                         to_dev(d["vclk"][:, k0:k1])[None], to_dev(d["vval"][:, k0:k1])[None],
                                         k0, 37, vout=8, **kw)
        np.testing.assert_array_equal(to_host(res.clock)[0], exp[0])
        np.testing.assert_array_equal(to_host(res.ec)[0], exp[1][k0:k1])
        np.testing.assert_array_equal(to_host(res.vclk)[0], exp[2][k0:k1])
        np.testing.assert_array_equal(to_host(res.vval)[0], exp[3][k0:k1])
        union = res.def_keys if union is None else union | res.def_keys
        keep = res.def_keep
    assert cg.map.deferred_set(kw["def_clock"], keep, union) == exp[5]
