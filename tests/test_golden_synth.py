"""The synthetic generators pinned by tests/golden/synth.json (written by
tests/golden/make_golden.py): the oracle's restatement (CPU) and the device generators (GPU)
must both reproduce the fixture, and the kernels must reproduce its folds."""
import json
import os

import numpy as np
import pytest

import oracle as O

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "synth.json")))


def arr(v, shape):
    return np.array([int(x) for x in v], dtype=np.uint64).reshape(shape)


def test_oracle_synth_fill_matches_fixture():
    for f in GOLD["fill"]:
        m = O.synth_matrix(f["seed"], f["rows"], f["width"], f["kind"], row0=f["first_row"])
        np.testing.assert_array_equal(m, arr(f["values"], (f["rows"], f["width"])))


def test_oracle_synth_orswot_matches_fixture():
    g = GOLD["orswot"]
    R, M, A = g["R"], g["M"], g["A"]
    c, e = O.synth_orswot(g["seed"], R, M, A, g["kmax"], row0=g["row0"])
    np.testing.assert_array_equal(c, arr(g["clock"], (R, A)))
    np.testing.assert_array_equal(e, arr(g["entries"], (R, M, A)))
    fc, fe = O.dense_orswot_join_fold(c, e)
    np.testing.assert_array_equal(fe, arr(g["fold_entries"], (M, A)))
    assert fe.any()  # the removal model leaves live dots after the fold


def test_oracle_synth_map_matches_fixture():
    g = GOLD["map"]
    R, K, A, V = g["R"], g["K"], g["A"], g["V"]
    dfr = O.synth_map_deferred(g["seed"], R, K, A, g["kmax"], p_def=g["p_def"])
    d = O.synth_map(g["seed"], R, K, A, V, g["kmax"], deferred=dfr)
    np.testing.assert_array_equal(d["clock"], arr(g["clock"], (R, A)))
    np.testing.assert_array_equal(d["ec"], arr(g["ec"], (R, K, A)))
    np.testing.assert_array_equal(d["vclk"], arr(g["vclk"], (R, K, V, A)))
    np.testing.assert_array_equal(d["vval"], arr(g["vval"], (R, K, V)))
    assert len(g["def_row"]) > 0


@pytest.mark.gpu
def test_gpu_synth_and_folds_match_fixture(gpu_ctx):
    import torch

    import crdts_gpu as cg
    from crdts_gpu import synth
    from gpu_util import to_dev, to_host
    for f in GOLD["fill"]:
        out = torch.empty((f["rows"], f["width"]), dtype=torch.int64, device="cuda:0")
        cg.synth_fill(gpu_ctx, out, f["seed"], f["kind"], first_row=f["first_row"])
        np.testing.assert_array_equal(to_host(out), arr(f["values"], (f["rows"], f["width"])))
    g = GOLD["orswot"]
    R, M, A = g["R"], g["M"], g["A"]
    inp = synth.orswot_replicas(gpu_ctx, R, M, A, seed=g["seed"], kmax=g["kmax"], first_row=g["row0"], p_def=0.0)
    np.testing.assert_array_equal(to_host(inp.clock), arr(g["clock"], (R, A)))
    np.testing.assert_array_equal(to_host(inp.entries), arr(g["entries"], (R, M, A)))
    res = cg.orswot.lub_many(inp.clock, inp.entries, ctx=gpu_ctx)
    np.testing.assert_array_equal(to_host(res.entries), arr(g["fold_entries"], (M, A)))
    np.testing.assert_array_equal(to_host(res.clock), arr(g["fold_clock"], (A,)))
    g = GOLD["map"]
    R, K, A, V = g["R"], g["K"], g["A"], g["V"]
    inp = synth.map_replicas(gpu_ctx, R, K, A, V, g["seed"], kmax=g["kmax"], p_def=g["p_def"])
    for nm, shp in (("clock", (R, A)), ("ec", (R, K, A)), ("vclk", (R, K, V, A)), ("vval", (R, K, V))):
        np.testing.assert_array_equal(to_host(getattr(inp, nm)), arr(g[nm], shp), err_msg=nm)
    D = len(g["def_row"])
    Kw = (K + 63) // 64
    res = cg.map.lub_many(inp.clock, inp.ec, inp.vclk, inp.vval, def_off=[0, D],
                          def_row=torch.from_numpy(arr(g["def_row"], (D,)).astype(np.int32)).cuda(),
                          def_clock=to_dev(arr(g["def_clock"], (D, A))), def_keys=to_dev(arr(g["def_keys"], (D, Kw))),
                          vout=4, ctx=gpu_ctx)
    np.testing.assert_array_equal(to_host(res.clock), arr(g["fold_clock"], (A,)))
    np.testing.assert_array_equal(to_host(res.ec), arr(g["fold_ec"], (K, A)))
    np.testing.assert_array_equal(to_host(res.vclk), arr(g["fold_vclk"], (K, 4, A)))
    np.testing.assert_array_equal(to_host(res.vval), arr(g["fold_vval"], (K, 4)))
