"""World-2 sharded lub through the REAL kernels (the multi-rank path had only run
with the oracle injected as the local fold).

A fresh child `torch.distributed.run --nproc-per-node 2` runs tests/dist_world2_worker.py: both
ranks on GPU 0, gloo exchange (RCCL refuses two ranks per GPU; the RCCL path of the same
exchange is crdt_*_lub_many_sharded, tested at world 1 in test_gpu_shard_abi.py), the local
folds in libcrdt_gpu.  Every rank's received result must equal the oracle's left fold of the
whole input: VClock / GCounter / PNCounter / GSet (max all-reduce, OR re-fold), LWWReg (state and
the GLOBAL first conflicting merge), Orswot (re-merge with every rank's deferred removes) and
Map<K, MVReg> (key shards).  Reference fold: test/orswot.rs:50-53, map.rs:141-219,
lwwreg.rs:84-98."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import dist_world2_data as D
import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def outs(tmp_path_factory):
    out = tmp_path_factory.mktemp("world2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "dist_world2_worker.py"), "--out", str(out)]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return [dict(np.load(out / f"rank{k}.npz")) for k in range(2)]


def test_world2_used_the_hip_library(outs):
    for o in outs:
        assert bytes(o["lib"]).decode().endswith("libcrdt_gpu.so")


@pytest.mark.parametrize("name", sorted(D.LATTICES))
def test_world2_lattices(outs, name):
    kind, G, R, W = D.LATTICES[name]
    full = D.lattice_input(name)
    fold = O.gset_fold if kind == "gset" else O.vclock_fold
    exp = np.stack([fold(full[g])[0] for g in range(G)])
    for o in outs:
        np.testing.assert_array_equal(o[name].reshape(G, W), exp)


def test_world2_lwwreg(outs):
    m, v = D.lww_input()
    for o in outs:
        for g in range(m.shape[0]):
            om, ov, of, _ = O.lwwreg_fold(m[g], v[g])
            fc = int(o["lww_conflict"][g])
            assert (int(o["lww_marker"][g]), int(o["lww_val"][g]), 2**64 - 1 if fc == -1 else fc) == (om, ov, of)
    assert any(int(x) != -1 for x in outs[0]["lww_conflict"])  # the conflict path is exercised


def test_world2_orswot(outs):
    clock, entries, off, dcl, dmem = D.orswot_input()
    oc, oe, odef, _ = O.orswot_fold(clock, entries, off, dcl, dmem)
    assert odef  # surviving deferred removes are exercised
    for o in outs:
        np.testing.assert_array_equal(o["orswot_clock"][0], oc)
        np.testing.assert_array_equal(o["orswot_entries"][0], oe)
        got = {(tuple(int(x) for x in dcl[d]), O.bitmap_members(o["orswot_def_members"][d]))
               for d in np.flatnonzero(o["orswot_keep"])}
        assert got == odef


def test_world2_map(outs):
    d = D.map_input()
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"],
                     D.MAP_VOUT)
    K = d["ec"].shape[1]
    assert exp[5]  # surviving removes are exercised
    ks = []
    for o in outs:
        k0 = int(o["map_k0"][0])
        n = o["map_ec"].shape[1]
        ks.append((k0, n))
        np.testing.assert_array_equal(o["map_clock"][0], exp[0])
        np.testing.assert_array_equal(o["map_ec"][0], exp[1][k0:k0 + n])
        np.testing.assert_array_equal(o["map_vclk"][0], exp[2][k0:k0 + n])
        np.testing.assert_array_equal(o["map_vval"][0], exp[3][k0:k0 + n])
        np.testing.assert_array_equal(o["map_nval"][0], exp[4][k0:k0 + n])
        got = {(tuple(int(x) for x in d["def_clock"][j]), O.bitmap_members(o["map_def_keys"][j]))
               for j in np.flatnonzero(o["map_keep"])}
        assert got == exp[5]
    assert sorted(ks)[0][0] == 0 and sum(n for _, n in ks) == K
