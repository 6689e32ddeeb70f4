"""GPU parity: Orswot lub_many is the reference's left fold for ANY input states (VERDICT r3
missing #1 / next #2), not only for states that keep the reference invariants (E <= C, unique dots).

Deserialized states (serde derive, /root/reference/src/orswot.rs:20) can hold entry dots above their
replica's clock.  There the per-cell join is not associative, so a slice-parallel fold could differ
from `acc = Orswot::new(); for r: acc.merge(r)` (orswot.rs:81-149).  The join kernel flags such
cells and re-folds the affected units in replica order (csrc/orswot.hip), the host-streamed mode
continues that fold chunk by chunk, and the sharded entry point folds the ranks in rank order when a
shard holds one (csrc/shard.hip; its world-2 run is in tests/test_gpu_dist_world2.py).  Every result
here is compared with the oracle's restated left fold (oracle/ref_fold.cpp) over per-replica
deferred offsets, the removes applied at their own step."""
import numpy as np
import pytest
import torch

import oracle as O
from dist_world2_data import adversarial_orswot
from gpu_util import to_dev, to_host

pytestmark = pytest.mark.gpu

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import host  # noqa: E402


def expected(clock, entries, off, dcl, dmem):
    kw = (off, dcl, dmem) if int(off[-1]) else ()
    return O.orswot_fold(clock, entries, *kw)[:3]


def check(got_c, got_e, keep, members, dcl, exp, lo=0, hi=None):
    oc, oe, odef = exp
    np.testing.assert_array_equal(got_c, oc)
    np.testing.assert_array_equal(got_e, oe)
    hi = dcl.shape[0] if hi is None else hi
    surv = set() if keep is None else {(tuple(int(x) for x in dcl[d]), O.bitmap_members(members[d]))
                                      for d in range(lo, hi) if keep[d]}
    assert surv == odef


def test_planted_case_breaks_a_tree():
    """The planted cells make the tree grouping wrong (so the tests below exercise the re-fold)."""
    clock, entries, *_ = adversarial_orswot(1, 40, 3, 2)
    c1, e1 = O.dense_orswot_join_fold(clock, entries)
    ca, ea = O.dense_orswot_join_fold(clock[:20], entries[:20])
    cb, eb = O.dense_orswot_join_fold(clock[20:], entries[20:])
    _, e2 = O.dense_orswot_join_fold(np.stack([ca, cb]), np.stack([ea, eb]))
    assert int(e1[0, 0]) == 0 and int(e2[0, 0]) == 1


# launch forms of the join: default slices (many replica slices per unit at these shapes), one
# workgroup per CU, UR 2 / 4 replicas in flight, 8 / 16 member rows per thread
@pytest.mark.parametrize("tune", ["", "obpc=1", "ounroll=2", "ounroll=4", "ompt=8", "ompt=16"])
@pytest.mark.parametrize("seed,R,M,A", [(1, 2000, 6, 8), (2, 300, 70, 9), (3, 5000, 3, 64), (4, 3, 5, 2)])
def test_orswot_lub_many_any_state(seed, R, M, A, tune):
    clock, entries, off, dcl, dmem = adversarial_orswot(seed, R, M, A)
    ctx = cg.Context(0)
    if tune:
        ctx.tune(tune)
    D = dcl.shape[0]
    kw = dict(def_off=[0, D], def_clock=to_dev(dcl), def_members=to_dev(dmem)) if D else {}
    res = cg.orswot.lub_many(to_dev(clock), to_dev(entries), ctx=ctx, **kw)
    keep = None if res.def_keep is None else res.def_keep.cpu().numpy()
    members = None if res.def_members is None else to_host(res.def_members)
    check(to_host(res.clock), to_host(res.entries), keep, members, dcl, expected(clock, entries, off, dcl, dmem))
    ctx.close()


def test_orswot_lub_many_any_state_groups_and_doff(gpu_ctx):
    """Several groups, some well-formed (no re-fold) and some not, with the deferred pool's offsets in
    host and in device memory: every group equals its own left fold."""
    G, R, M, A = 5, 700, 9, 8
    parts = [adversarial_orswot(50 + g, R, M, A, plant=g % 2 == 0) if g != 3 else
             O.gen_orswot(50 + g, R, M, A, kmax=10, p_def=0.3) for g in range(G)]
    clock = np.stack([p[0] for p in parts])
    entries = np.stack([p[1] for p in parts])
    dcl = np.concatenate([p[3] for p in parts])
    dmem = np.concatenate([p[4] for p in parts])
    goff = np.cumsum([0] + [p[3].shape[0] for p in parts]).astype(np.int64)
    for form in ("host_off", "device_off"):
        st = torch.full((1,), -1, dtype=torch.int32, device="cuda:0")
        off = goff if form == "host_off" else torch.from_numpy(goff).cuda()
        kw = dict(def_status=st) if form == "device_off" else {}
        res = cg.orswot.lub_many(to_dev(clock), to_dev(entries), def_off=off, def_clock=to_dev(dcl),
                                 def_members=to_dev(dmem), ctx=gpu_ctx, **kw)
        keep, members = res.def_keep.cpu().numpy(), to_host(res.def_members)
        gc, ge = to_host(res.clock), to_host(res.entries)
        for g, p in enumerate(parts):
            check(gc[g], ge[g], keep, members, dcl, expected(*p), int(goff[g]), int(goff[g + 1]))
        if form == "device_off":
            assert int(st.item()) == 0


@pytest.mark.parametrize("stage_kb,R", [(8, 300), (64, 2000), (1 << 18, 2000)])
def test_orswot_host_streamed_any_state(stage_kb, R):
    """CRDT_MEM_HOST: replica chunks joined behind the running join (slot 0) — the planted cells
    straddle chunk boundaries at the small stage sizes — streamed and whole-batch both exact."""
    clock, entries, off, dcl, dmem = adversarial_orswot(7 + R, R, 12, 8)
    D = dcl.shape[0]
    exp = expected(clock, entries, off, dcl, dmem)
    for hs in (1, 0):
        ctx = host.HostContext(0, tune=f"stage_kb={stage_kb},hstream={hs}")
        got = host.orswot_lub_many(clock[None], entries[None], def_off=[0, D], def_clock=dcl, def_members=dmem,
                                   ctx=ctx)
        ctx.close()
        check(got.clock[0], got.entries[0], got.def_keep, got.def_members, dcl, exp)


def test_orswot_sharded_world1_any_state():
    """crdt_orswot_lub_many_sharded at world 1 on arbitrary states (the local join re-folds in order;
    the rank-order chain itself needs two ranks: tests/test_gpu_dist_world2.py)."""
    clock, entries, off, dcl, dmem = adversarial_orswot(99, 1500, 10, 8)
    ctx = cg.Context(0)
    cg.shard.comm_init(ctx, cg.shard.unique_id(), 1, 0)
    D = dcl.shape[0]
    res = cg.shard.orswot_lub_many_sharded(to_dev(clock[None]), to_dev(entries[None]), def_off=[0, D],
                                           def_clock=to_dev(dcl), def_members=to_dev(dmem), ctx=ctx)
    oc, oe, odef = expected(clock, entries, off, dcl, dmem)
    np.testing.assert_array_equal(to_host(res.clock)[0], oc)
    np.testing.assert_array_equal(to_host(res.entries)[0], oe)
    assert cg.shard.deferred_groups(res, 1)[0] == odef
    cg.shard.comm_destroy(ctx)
    ctx.close()
