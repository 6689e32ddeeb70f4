"""GPU parity at the BASELINE sizes themselves (configs 3 and 4 had only run at full
size in builder logs).

Config 3: Orswot<u64, u32> lub of 65,536 replicas x 4,096 members x 64 actors (128 GiB of
entries in HBM) with ~13k deferred removes.  Config 4: Map<u32, MVReg<u64>> lub of 16,384
replicas x 1,024 keys x 32 actors, V = 2.  Inputs are generated in HBM by crdt_synth_* and
regenerated on the CPU by the oracle's independent restatement (checked on the sample).

The merge is independent per member (Orswot) / per key (Map) given the replica clocks and the
deferred list, so the oracle's fold over EVERY replica restricted to 64 sampled members / keys
must equal the GPU result restricted to them.  The surviving deferred removes are checked whole:
every survivor's clock and its complete member set (Orswot), and every survivor with its key set
restricted to the sample (Map).  Reference fold: test/orswot.rs:50-53, orswot.rs:81-149,
map.rs:141-219."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import synth  # noqa: E402

u64 = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731


def test_config3_orswot_full_size(gpu_ctx):
    R, M, A, kmax, seed = 65536, 4096, 64, 48, 0x5EED0003
    inp = synth.orswot_replicas(gpu_ctx, R, M, A, seed=seed, kmax=kmax, p_def=0.1)
    D = inp.def_clock.shape[0]
    res = cg.orswot.lub_many(inp.clock, inp.entries, def_off=[0, D], def_clock=inp.def_clock,
                             def_members=inp.def_members, ctx=gpu_ctx)
    torch.cuda.synchronize()
    msub = np.sort(np.random.default_rng(3).choice(M, size=64, replace=False))
    tsub = torch.from_numpy(msub).cuda()
    clock_h = u64(inp.clock)
    ent_h = u64(inp.entries[:, tsub, :].contiguous())
    got_c, got_e = u64(res.clock), u64(res.entries[tsub])
    keep, gmem = res.def_keep.cpu().numpy(), u64(res.def_members)
    dcl_h, dmem_h = u64(inp.def_clock), u64(inp.def_members)
    def_off = inp.def_off
    del inp, res
    torch.cuda.empty_cache()
    # the device generator agrees with the CPU restatement (replica rows incl. their applied removes)
    drow = np.repeat(np.arange(R), np.diff(def_off.astype(np.int64)))
    for r in (0, 12345, R - 1) + tuple(drow[:2]):
        c_cpu, e_cpu = O.synth_orswot(seed, 1, M, A, kmax, row0=int(r))
        dr = np.flatnonzero(drow == r)
        e_cpu = O.apply_rm_rows(e_cpu, [0] * len(dr), dcl_h[dr], dmem_h[dr])
        assert np.array_equal(c_cpu[0], clock_h[r])
        assert np.array_equal(e_cpu[0][msub], ent_h[r])
    sub_mem = np.zeros((D, 1), np.uint64)
    for j, m in enumerate(msub):
        sub_mem[:, 0] |= ((dmem_h[:, m // 64] >> np.uint64(m % 64)) & np.uint64(1)) << np.uint64(j)
    oc, oe, odef_sub = O.dense_orswot_lub(clock_h, ent_h, dcl_h, sub_mem)
    np.testing.assert_array_equal(got_c, oc)
    np.testing.assert_array_equal(got_e, oe)
    assert oe.any() and D > 10000
    # every surviving deferred remove, with its whole member set
    exp_def = O.dense_orswot_survivors(oc, dcl_h, dmem_h)
    got_def = {(tuple(int(x) for x in dcl_h[d]), O.bitmap_members(gmem[d])) for d in np.flatnonzero(keep)}
    assert len(exp_def) > 1000
    assert got_def == exp_def


def test_config4_map_full_size(gpu_ctx):
    R, K, A, V, kmax, seed, vout = 16384, 1024, 32, 2, 256, 0x5EED0004, 4
    inp = synth.map_replicas(gpu_ctx, R, K, A, V, seed, kmax=kmax, p_def=0.1)
    # the synthetic removes are all dominated by the final clock: add 40 from the far future (never
    # dominated) so surviving removes and their key unions are checked too (exact for any input)
    rng = np.random.default_rng(4)
    rows = np.concatenate([inp.def_row.cpu().numpy().astype(np.int64), rng.integers(0, R, size=40)])
    extra = np.zeros((40, A), np.uint64)
    extra[np.arange(40), rng.integers(0, A, size=40)] = np.uint64(10**9) + np.arange(40, dtype=np.uint64) % 7
    ekeys = np.zeros((40, K // 64), np.uint64)
    for j in range(40):
        for k in rng.choice(K, size=int(rng.integers(1, 50)), replace=False):
            ekeys[j, k // 64] |= np.uint64(1) << np.uint64(k % 64)
    dcl = np.concatenate([u64(inp.def_clock), extra])
    dks = np.concatenate([u64(inp.def_keys), ekeys])
    order = np.argsort(rows, kind="stable")
    rows, dcl, dks = rows[order], dcl[order], dks[order]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()  # noqa: E731
    Dn = rows.shape[0]
    res = cg.map.lub_many(inp.clock, inp.ec, inp.vclk, inp.vval, def_off=[0, Dn],
                          def_row=torch.from_numpy(rows.astype(np.int32)).cuda(), def_clock=t(dcl),
                          def_keys=t(dks), vout=vout, ctx=gpu_ctx)
    # the one- and two-wave (mst) forms of the A = 32, V = 2 fold agree on the whole result
    for spec in ("mst=0", "mst=1"):
        alt = cg.Context(0)
        alt.tune(spec)
        res2 = cg.map.lub_many(inp.clock, inp.ec, inp.vclk, inp.vval, def_off=[0, Dn],
                               def_row=torch.from_numpy(rows.astype(np.int32)).cuda(), def_clock=t(dcl),
                               def_keys=t(dks), vout=vout, ctx=alt)
        torch.cuda.synchronize()
        for nm in ("clock", "ec", "vclk", "vval", "nval", "flags", "def_keep", "def_keys"):
            assert torch.equal(getattr(res, nm), getattr(res2, nm)), (spec, nm)
        del res2
        alt.close()
    keys = np.sort(np.random.default_rng(5).choice(K, size=64, replace=False))
    tk = torch.from_numpy(keys).cuda()
    dev = {nm: u64(getattr(inp, nm) if nm == "clock" else getattr(inp, nm)[:, tk]) for nm in ("clock", "ec", "vclk", "vval")}
    got = dict(clock=u64(res.clock), ec=u64(res.ec)[keys], vclk=u64(res.vclk)[keys], vval=u64(res.vval)[keys],
               nval=res.nval.cpu().numpy()[keys], flags=int(res.flags.cpu().numpy().max()))
    keep, gkeys = res.def_keep.cpu().numpy(), u64(res.def_keys)
    del inp, res
    torch.cuda.empty_cache()
    # the device generator agrees with the CPU restatement on the sample
    dfr = O.synth_map_deferred(seed, R, K, A, kmax, p_def=0.1)
    d = O.synth_map(seed, R, K, A, V, kmax, keys=keys, deferred=dfr)
    for nm in ("clock", "ec", "vclk", "vval"):
        np.testing.assert_array_equal(dev[nm], d[nm], err_msg=nm)
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], rows, dcl, O.restrict_deferred_keys(dks, keys), vout)
    assert got["flags"] == 0
    np.testing.assert_array_equal(got["clock"], exp[0])
    np.testing.assert_array_equal(got["ec"], exp[1])
    np.testing.assert_array_equal(got["vclk"], exp[2])
    np.testing.assert_array_equal(got["vval"], exp[3])
    np.testing.assert_array_equal(got["nval"], exp[4])
    assert exp[4].any() and (exp[4] == 2).any()
    # every surviving remove (clock), with its key set restricted to the sample
    pos = {int(k): i for i, k in enumerate(keys)}
    got_def = {}
    for j in np.flatnonzero(keep):
        sub = frozenset(pos[k] for k in O.bitmap_members(gkeys[j]) if k in pos)
        got_def[tuple(int(x) for x in dcl[j])] = sub
    exp_def = {c: ks for c, ks in exp[5]}
    assert set(got_def) >= set(exp_def) and len(got_def) >= 30
    assert {c: ks for c, ks in got_def.items() if ks} == {c: ks for c, ks in exp_def.items() if ks}
    # a survivor with no key in the sample is absent from the restricted oracle fold; its
    # survival is still !(rm <= final clock)
    for c in set(got_def) - set(exp_def):
        assert got_def[c] == frozenset() and np.any(np.array(c, np.uint64) > exp[0])
