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
    ranks = "\n".join(x for x in r.stderr.splitlines() if x.startswith("[rank") or "Error" in x or "File " in x)
    assert r.returncode == 0, ranks[-6000:] + "\n" + r.stdout[-2000:] + r.stderr[-2000:]
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


# ---- the C ABI's own multi-rank code (csrc/shard.hip) through crdt_ctx_comm_init_ops -------------
def test_world2_cabi_comm(outs):
    for k, o in enumerate(outs):
        assert tuple(o["cabi_comm"]) == (2, k)


@pytest.mark.parametrize("name", sorted(D.LATTICES))
def test_world2_cabi_lattices(outs, name):
    kind, G, R, W = D.LATTICES[name]
    full = D.lattice_input(name)
    fold = O.gset_fold if kind == "gset" else O.vclock_fold
    exp = np.stack([fold(full[g])[0] for g in range(G)])
    for o in outs:
        np.testing.assert_array_equal(o["cabi_" + name].reshape(G, W), exp)
        np.testing.assert_array_equal(o["cabi_multi_" + name].reshape(G, W), exp)


@pytest.mark.parametrize("tag", ["even", "r0empty", "uneven"])
def test_world2_cabi_lwwreg(outs, tag):
    """crdt_lwwreg_lub_many_sharded at world 2: the state and the GLOBAL first conflicting merge,
    incl. a rank holding no replica (the "lower non-empty ranks" prefix, shard.hip)."""
    m, v = D.lww_input()
    for o in outs:
        for g in range(m.shape[0]):
            om, ov, of, _ = O.lwwreg_fold(m[g], v[g])
            fc = int(o[f"cabi_lww_{tag}_conflict"][g])
            got = (int(o[f"cabi_lww_{tag}_marker"][g]), int(o[f"cabi_lww_{tag}_val"][g]), 2**64 - 1 if fc == -1 else fc)
            assert got == (om, ov, of)
    assert any(int(x) != -1 for x in outs[0][f"cabi_lww_{tag}_conflict"])


def test_world2_cabi_orswot(outs):
    """crdt_orswot_lub_many_sharded at world 2: both ranks hold deferred removes, so the regroup
    (rank order, then local order: r*Dmax + base[r]) and the compaction are exercised."""
    clock, entries, off, dcl, dmem = D.orswot_input()
    oc, oe, odef, _ = O.orswot_fold(clock, entries, off, dcl, dmem)
    assert odef and all(int(o["cabi_orswot_ndef_local"][0]) > 0 for o in outs)
    for o in outs:
        np.testing.assert_array_equal(o["cabi_orswot_clock"][0], oc)
        np.testing.assert_array_equal(o["cabi_orswot_entries"][0], oe)
        got = {(tuple(int(x) for x in o["cabi_orswot_def_clock"][d]), O.bitmap_members(o["cabi_orswot_def_members"][d]))
               for d in range(o["cabi_orswot_def_clock"].shape[0])}
        assert got == odef


def test_world2_cabi_orswot_doff(outs):
    """crdt_orswot_lub_many_sharded_doff at world 2: the same result as the host-offset call (device
    counts in the exchanged row); invalid offsets on rank 1 only -> EINVAL there, ECOMM on rank 0."""
    for o in outs:
        for k in ("clock", "entries", "def_clock", "def_members"):
            np.testing.assert_array_equal(o[f"cabi_orswot_doff_{k}"], o[f"cabi_orswot_{k}"])
    codes = sorted(int(o["cabi_orswot_badoff_code"][0]) for o in outs)
    assert codes == sorted([-1, -5]), codes  # CRDT_EINVAL, CRDT_ECOMM


def test_world2_cabi_map_offsets_differ(outs):
    """Device offsets that differ between the ranks (same G and D): both ranks return EINVAL."""
    assert all(int(o["cabi_mapoff_code"][0]) == -1 for o in outs)  # CRDT_EINVAL


def test_world2_cabi_orswot_any_state(outs):
    """crdt_orswot_lub_many_sharded at world 2 on states with E > C cells whose non-associative
    sequence spans the rank boundary: the ranks fold in rank order (csrc/shard.hip), so both hold
    the reference's left fold, not the tree join of the rank partials."""
    clock, entries, off, dcl, dmem = D.orswot_any_input()
    kw = (off, dcl, dmem) if int(off[-1]) else ()
    oc, oe, odef, _ = O.orswot_fold(clock, entries, *kw)
    assert int(oe[0, 0]) == 0  # the planted dot: dropped by the left fold, kept by a tree
    for o in outs:
        np.testing.assert_array_equal(o["cabi_orswot_any_clock"][0], oc)
        np.testing.assert_array_equal(o["cabi_orswot_any_entries"][0], oe)
        got = {(tuple(int(x) for x in o["cabi_orswot_any_def_clock"][d]),
                O.bitmap_members(o["cabi_orswot_any_def_members"][d]))
               for d in range(o["cabi_orswot_any_def_clock"].shape[0])}
        assert got == odef


@pytest.mark.parametrize("tag", ["even", "empty", "even_doff", "empty_doff"])
def test_world2_cabi_map(outs, tag):
    """crdt_map_lub_many_sharded at world 2: key placement at k0 != 0 with the SUM all-reduce, and
    a rank whose key shard is EMPTY (it must still join every collective: ADVICE r2)."""
    d = D.map_input()
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"],
                     D.MAP_VOUT)
    assert exp[5]
    covered = []
    for o in outs:
        k0, k1 = (int(x) for x in o[f"cabi_map_{tag}_k0"])
        covered.append((k0, k1))
        np.testing.assert_array_equal(o[f"cabi_map_{tag}_clock"][0], exp[0])
        np.testing.assert_array_equal(o[f"cabi_map_{tag}_ec"][0], exp[1][k0:k1])
        np.testing.assert_array_equal(o[f"cabi_map_{tag}_vclk"][0], exp[2][k0:k1])
        np.testing.assert_array_equal(o[f"cabi_map_{tag}_vval"][0], exp[3][k0:k1])
        np.testing.assert_array_equal(o[f"cabi_map_{tag}_nval"][0], exp[4][k0:k1])
        got = {(tuple(int(x) for x in d["def_clock"][j]), O.bitmap_members(o[f"cabi_map_{tag}_def_keys"][j]))
               for j in np.flatnonzero(o[f"cabi_map_{tag}_keep"])}
        assert got == exp[5]
    if tag.startswith("empty"):
        assert (d["ec"].shape[1], d["ec"].shape[1]) in covered


@pytest.mark.parametrize("tag,names", [("c1", ("clock", "ec", "val", "keep", "keys", "flags")),
                                       ("c2", ("clock", "ec", "val", "keep", "keys", "flags")),
                                       ("o", ("clock", "ec", "oc", "ent", "keep", "keys", "flags"))])
def test_world2_cabi_value_maps(outs, tag, names):
    """crdt_map_counter_lub_many_sharded (W = 1, 2) and crdt_map_orswot_lub_many_sharded at world 2
    (round 5): each rank's keys equal the same rank's unsharded fold of every key restricted to them,
    and the surviving removes' key sets after the SUM all-reduce equal the unsharded fold's over ALL
    keys (the two key ranges cover K).  The unsharded folds are parity-tested against the oracle in
    tests/test_gpu_map_counter.py / test_gpu_map_orswot.py."""
    K = D.map_input()["ec"].shape[1]
    covered = set()
    for o in outs:
        k0, k1 = (int(x) for x in o[f"vmap_{tag}_k0"])
        covered |= set(range(k0, k1))
        for nm in names:
            if f"vmap_{tag}_full_{nm}" in o:
                np.testing.assert_array_equal(o[f"vmap_{tag}_sh_{nm}"], o[f"vmap_{tag}_full_{nm}"], err_msg=nm)
        assert f"vmap_{tag}_sh_keys" in o  # (the input holds surviving removes)
    assert covered == set(range(K))


def test_world2_cabi_map_overflow_on_one_rank(outs):
    """Only rank 1's key folds to 12 values: with vout=8 its fold state (8 values) overflows, the C
    call reruns EVERY rank with the 16-value state (the retry used to be rank-local, so
    one rank entered the collective twice), and the global flags make BOTH ranks raise the capacity
    error; with vout=16 both return the exact fold."""
    assert all(int(o["cabi_mapovf_raised"][0]) == 1 for o in outs)
    d = D.map_overflow_input()
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"],
                     D.MAP_OVF_VOUT)
    assert int(exp[4][-1]) == 12
    for o in outs:
        k0, k1 = (int(x) for x in o["cabi_mapovf_k0"])
        np.testing.assert_array_equal(o["cabi_mapovf_ec"][0], exp[1][k0:k1])
        np.testing.assert_array_equal(o["cabi_mapovf_vclk"][0], exp[2][k0:k1])
        np.testing.assert_array_equal(o["cabi_mapovf_vval"][0], exp[3][k0:k1])
        np.testing.assert_array_equal(o["cabi_mapovf_nval"][0], exp[4][k0:k1])
    assert int(outs[0]["cabi_mapovf_flags"][0]) == int(outs[1]["cabi_mapovf_flags"][0])


def test_world2_cabi_map_vstate_mismatch(outs):
    """Rank 0 starts the fold with a 16-value state, rank 1 with none, and a key overflows the
    smaller one: the overflow retry branches on the state size, so a mismatch must be refused on
    EVERY rank (EINVAL) before the collectives instead of leaving the ranks in different ones."""
    EINVAL = -1
    for o in outs:
        assert int(o["cabi_mapvstate_code"][0]) == EINVAL


def test_world2_cabi_errors_agree(outs):
    """A NULL output on rank 1 (its own validation fails) and a row width that differs between the
    ranks: no rank blocks, every rank reports an error.  On a plan the ranks agreed earlier (no header
    exchange, csrc/shard_host.hpp PlanCache) rank 1 errs in the call and every rank reports ECOMM at its
    next sharded call; the plans are then forgotten and the width mismatch errs on both ranks in the
    call; with shagree=1 both errors come in the call itself.  Afterwards the communicator works: one
    header exchange for three good calls, the last two on the agreed plan, all equal to the oracle fold."""
    EINVAL, ECOMM = -1, -5
    assert tuple(outs[0]["cabi_error_codes"]) == (0, ECOMM, EINVAL)
    assert tuple(outs[1]["cabi_error_codes"]) == (EINVAL, ECOMM, EINVAL)
    assert tuple(outs[0]["cabi_error_codes_sync"]) == (ECOMM, EINVAL)
    assert tuple(outs[1]["cabi_error_codes_sync"]) == (EINVAL, EINVAL)
    exp = O.vclock_fold(D.lattice_input("vclock")[0])[0]
    for o in outs:
        np.testing.assert_array_equal(o["cabi_pre_errors"], exp)
        np.testing.assert_array_equal(o["cabi_after_errors"], exp)
        for r in o["cabi_after_errors_cached"]:
            np.testing.assert_array_equal(r, exp)
        assert tuple(o["cabi_agree_calls"]) == (1, 3)  # one header exchange, three data exchanges


def test_world2_cabi_config5(outs):
    """Config 5 at world 2 through the C ABI's own sharded entry point (the callback seam: RCCL
    refuses two ranks on one GPU): 2 x 1,048,576 VClock replicas x 1,024 actors.  Sampled actor
    columns equal the oracle's left fold of VClock::merge over ALL 2M replicas; every column equals
    the max of the two ranks' local maxima; both ranks hold the same result."""
    assert (D.C5_R, D.C5_A, D.C5_SEED) == (1 << 20, 1024, 0x5EED0005)
    exp_cols = D.c5_expected_columns(2 * D.C5_R)
    full = np.maximum(outs[0]["cabi_c5_local_max"], outs[1]["cabi_c5_local_max"])
    for o in outs:
        np.testing.assert_array_equal(o["cabi_c5"][D.C5_COLS], exp_cols)
        np.testing.assert_array_equal(o["cabi_c5"], full)
        lub_ms, xch_ms, agr_ms = (float(v) for v in o["cabi_c5_timing_ms"])
        assert lub_ms > 0 and xch_ms > 0 and agr_ms > 0  # the library timed every phase
    assert not np.array_equal(outs[0]["cabi_c5_local_max"], outs[1]["cabi_c5_local_max"])
