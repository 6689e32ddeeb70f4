"""One rank of the world-2 sharded-lub check with the REAL kernels (run by
tests/test_gpu_dist_world2.py through torch.distributed.run; not a test module itself).

Every rank builds the same seeded global input, keeps its own shard (dist.shard_range), runs the
crdts_gpu.dist sharded entry points with libcrdt_gpu as the local fold (nothing injected), and
saves what it received to <out>/rank<r>.npz.  The parent test compares every rank's output with
the oracle's fold of the whole input.  Both ranks sit on GPU 0 and exchange over gloo (RCCL
refuses two ranks on one GPU); gloo collectives of device tensors are staged through host
memory by crdts_gpu.dist."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "rust-crdt_amd"), os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dist_world2_data as D  # noqa: E402


def main():
    try:
        _main()
    except BaseException:
        import traceback
        traceback.print_exc()
        sys.stderr.flush()
        raise


def _main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import crdts_gpu as cg
    from crdts_gpu import dist as cdist

    dev = "cuda:0"
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64).copy()).to(dev)  # noqa: E731
    h = lambda x: x.detach().cpu().numpy().view(np.uint64).copy()  # noqa: E731
    out = {}
    # four lattices: local lub_many kernel + MAX all-reduce (OR re-fold for GSet)
    for name, (kind, G, R, W) in D.LATTICES.items():
        full = D.lattice_input(name)
        lo, hi = cdist.shard_range(R, rank, world)
        shard = t(full[:, lo:hi])
        if G == 1:
            shard = shard[0]
        out[name] = h(cdist.lub_many_sharded(kind, shard))
    # LWWReg: exact first conflict of the GLOBAL left fold
    m, v = D.lww_input()
    lo, hi = cdist.shard_range(m.shape[1], rank, world)
    fm, fv, fc = cdist.lwwreg_lub_many_sharded(t(m[:, lo:hi]), t(v[:, lo:hi]), lo)
    out["lww_marker"], out["lww_val"] = h(fm), h(fv)
    out["lww_conflict"] = fc.cpu().numpy().copy()
    # Orswot: join of each shard without removes, all-gather + re-merge with every deferred remove
    clock, entries, off, dcl, dmem = D.orswot_input()
    R = clock.shape[0]
    lo, hi = cdist.shard_range(R, rank, world)
    d0, d1 = int(off[lo]), int(off[hi])
    res = cdist.orswot_lub_many_sharded(t(clock[lo:hi][None]), t(entries[lo:hi][None]), t(dcl[d0:d1]),
                                        t(dmem[d0:d1]), torch.zeros(d1 - d0, dtype=torch.int64, device=dev))
    out["orswot_clock"], out["orswot_entries"] = h(res.clock), h(res.entries)
    # the re-merge pools removes in rank order, then local order == the input order here
    out["orswot_keep"] = res.def_keep.cpu().numpy().copy()
    out["orswot_def_members"] = h(res.def_members)
    # Map<K, MVReg>: key shards, exact left fold per key, SUM all-reduce of surviving-remove key sets
    d = D.map_input()
    K = d["ec"].shape[1]
    k0, k1 = cdist.shard_range(K, rank, world)
    Dn = d["def_row"].shape[0]
    kw = dict(def_off=[0, Dn], def_row=torch.from_numpy(d["def_row"].astype(np.int32)).to(dev),
              def_clock=t(d["def_clock"]), def_keys=t(d["def_keys"])) if Dn else {}
    mres = cdist.map_lub_many_sharded(t(d["clock"][None]), t(d["ec"][None, :, k0:k1]), t(d["vclk"][None, :, k0:k1]),
                                      t(d["vval"][None, :, k0:k1]), k0, K, vout=D.MAP_VOUT, **kw)
    out["map_k0"] = np.array([k0], np.int64)
    out["map_clock"], out["map_ec"], out["map_vclk"], out["map_vval"] = (h(mres.clock), h(mres.ec), h(mres.vclk),
                                                                         h(mres.vval))
    out["map_nval"] = mres.nval.cpu().numpy().copy()
    out["map_keep"] = mres.def_keep.cpu().numpy().copy()
    out["map_def_keys"] = h(mres.def_keys)
    out.update(cabi_seam(rank, world, t, h))
    out["lib"] = np.frombuffer(cg._abi.LIB_PATH.encode(), np.uint8)
    torch.cuda.synchronize()
    np.savez(os.path.join(args.out, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


def cabi_seam(rank, world, t, h):
    """The C ABI's own multi-rank code (csrc/shard.hip: agreement, regrouping, LWW prefix, Map key
    placement and overflow retry) at world 2 through crdt_ctx_comm_init_ops: the exchange runs over
    gloo host callbacks instead of RCCL (RCCL refuses two ranks on one GPU)."""
    import crdts_gpu as cg
    from crdts_gpu import dist as cdist
    from crdts_gpu import shard as cs
    from crdts_gpu._abi import CrdtGpuError

    dev = "cuda:0"
    ctx = cg.Context(0)
    cs.comm_init_ops(ctx, cs.TorchCommOps(), world, rank)
    o = {"cabi_comm": np.array(cs.comm_info(ctx), np.int64)}
    for name, (kind, G, R, W) in D.LATTICES.items():
        full = D.lattice_input(name)
        lo, hi = cdist.shard_range(R, rank, world)
        shard = t(full[:, lo:hi])
        if G == 1:
            shard = shard[0]
        o["cabi_" + name] = h(cs.lub_many_sharded(kind, shard, ctx=ctx))
    # fused: every lattice of the step in one local launch + one grouped exchange
    items = []
    for name, (kind, G, R, W) in D.LATTICES.items():
        full = D.lattice_input(name)
        lo, hi = cdist.shard_range(R, rank, world)
        sh = t(full[:, lo:hi])
        items.append((kind, sh, torch.empty((G, W), dtype=torch.int64, device=dev)))
    cs.lub_many_multi_sharded(items, ctx=ctx)
    for (_, _, ob), name in zip(items, D.LATTICES):
        o["cabi_multi_" + name] = h(ob)
    # LWWReg: even split, and rank 0 holding NO replica (the lower-non-empty-ranks prefix)
    m, v = D.lww_input()
    Rl = m.shape[1]
    for tag, (lo, hi) in (("even", cdist.shard_range(Rl, rank, world)),
                          ("r0empty", (0, 0) if rank == 0 else (0, Rl)),
                          ("uneven", (0, 13) if rank == 0 else (13, Rl))):
        fm, fv, fc = cs.lwwreg_lub_many_sharded(t(m[:, lo:hi]), t(v[:, lo:hi]), lo, ctx=ctx)
        o[f"cabi_lww_{tag}_marker"], o[f"cabi_lww_{tag}_val"] = h(fm), h(fv)
        o[f"cabi_lww_{tag}_conflict"] = fc.cpu().numpy().copy()
    # Orswot: each rank's removes pooled per group; the regroup is rank order, then local order
    clock, entries, off, dcl, dmem = D.orswot_input()
    R = clock.shape[0]
    lo, hi = cdist.shard_range(R, rank, world)
    d0, d1 = int(off[lo]), int(off[hi])
    kw = dict(def_off=[0, d1 - d0], def_clock=t(dcl[d0:d1]), def_members=t(dmem[d0:d1])) if d1 > d0 else {}
    res = cs.orswot_lub_many_sharded(t(clock[lo:hi][None]), t(entries[lo:hi][None]), ctx=ctx, **kw)
    o["cabi_orswot_clock"], o["cabi_orswot_entries"] = h(res.clock), h(res.entries)
    o["cabi_orswot_def_clock"], o["cabi_orswot_def_members"] = h(res.def_clock), h(res.def_members)
    o["cabi_orswot_ndef_local"] = np.array([d1 - d0], np.int64)
    # the same with the offsets in device memory (crdt_orswot_lub_many_sharded_doff: counts taken on
    # the device, no host copy of the offsets)
    if d1 > d0:
        kw["def_off"] = torch.tensor([0, d1 - d0], dtype=torch.int64, device=dev)
    res = cs.orswot_lub_many_sharded(t(clock[lo:hi][None]), t(entries[lo:hi][None]), ctx=ctx, **kw)
    o["cabi_orswot_doff_clock"], o["cabi_orswot_doff_entries"] = h(res.clock), h(res.entries)
    o["cabi_orswot_doff_def_clock"], o["cabi_orswot_doff_def_members"] = h(res.def_clock), h(res.def_members)
    # invalid device offsets on rank 1 only: rank 1 gets EINVAL, rank 0 ECOMM, nobody blocks
    Dl = max(d1 - d0, 1)
    bad_off = torch.tensor([0, Dl] if rank == 0 else [1, Dl], dtype=torch.int64, device=dev)
    zc = torch.zeros((Dl, clock.shape[1]), dtype=torch.int64, device=dev)
    zm = torch.zeros((Dl, dmem.shape[1]), dtype=torch.int64, device=dev)
    try:
        cs.orswot_lub_many_sharded(t(clock[lo:hi][None]), t(entries[lo:hi][None]), bad_off, zc, zm, ctx=ctx)
        o["cabi_orswot_badoff_code"] = np.array([0], np.int64)
    except CrdtGpuError as e:
        o["cabi_orswot_badoff_code"] = np.array([e.code], np.int64)
    # Orswot on ARBITRARY states (E > C cells): the planted non-associative cells sit
    # at replica 0 (rank 0) and R-2, R-1 (rank 1), so joining the rank partials as a tree is wrong; the
    # flags gathered with the deferred counts switch the ranks to the rank-order chain
    clock, entries, off, dcl, dmem = D.orswot_any_input()
    R = clock.shape[0]
    lo, hi = cdist.shard_range(R, rank, world)
    d0, d1 = int(off[lo]), int(off[hi])
    kw = dict(def_off=[0, d1 - d0], def_clock=t(dcl[d0:d1]), def_members=t(dmem[d0:d1])) if d1 > d0 else {}
    res = cs.orswot_lub_many_sharded(t(clock[lo:hi][None]), t(entries[lo:hi][None]), ctx=ctx, **kw)
    o["cabi_orswot_any_clock"], o["cabi_orswot_any_entries"] = h(res.clock), h(res.entries)
    o["cabi_orswot_any_def_clock"], o["cabi_orswot_any_def_members"] = h(res.def_clock), h(res.def_members)
    # Map<K, MVReg>: key shards (k0 != 0 on rank 1), then an EMPTY key shard on rank 1
    d = D.map_input()
    K = d["ec"].shape[1]
    Dn = d["def_row"].shape[0]
    kw = dict(def_off=[0, Dn], def_row=torch.from_numpy(d["def_row"].astype(np.int32)).to(dev),
              def_clock=t(d["def_clock"]), def_keys=t(d["def_keys"])) if Dn else {}
    for tag, (k0, k1) in (("even", cdist.shard_range(K, rank, world)), ("empty", (0, K) if rank == 0 else (K, K)),
                          ("even_doff", cdist.shard_range(K, rank, world)),
                          ("empty_doff", (0, K) if rank == 0 else (K, K))):
        kwt = dict(kw)
        if tag.endswith("_doff") and Dn:  # offsets in device memory (crdt_map_lub_many_sharded_doff)
            kwt["def_off"] = torch.tensor([0, Dn], dtype=torch.int64, device=dev)
        mres = cs.map_lub_many_sharded(t(d["clock"][None]), t(d["ec"][None, :, k0:k1]), t(d["vclk"][None, :, k0:k1]),
                                       t(d["vval"][None, :, k0:k1]), k0, K, vout=D.MAP_VOUT, ctx=ctx, **kwt)
        o[f"cabi_map_{tag}_k0"] = np.array([k0, k1], np.int64)
        o[f"cabi_map_{tag}_clock"], o[f"cabi_map_{tag}_ec"] = h(mres.clock), h(mres.ec)
        o[f"cabi_map_{tag}_vclk"], o[f"cabi_map_{tag}_vval"] = h(mres.vclk), h(mres.vval)
        o[f"cabi_map_{tag}_nval"] = mres.nval.cpu().numpy().copy()
        o[f"cabi_map_{tag}_keep"] = mres.def_keep.cpu().numpy().copy()
        o[f"cabi_map_{tag}_def_keys"] = h(mres.def_keys)
    # value-typed Maps (round 5): key shards of Map<K, GCounter / PNCounter> (the MVReg input's value
    # clocks as counter rows) and Map<K, Orswot> (entry clock as the nested clock, value clocks as
    # member dots); each rank also folds every key unsharded (no collective) for the check
    k0, k1 = cdist.shard_range(K, rank, world)
    vc = d["vclk"]
    if vc.shape[2] < 2:
        vc = np.concatenate([vc, np.zeros(vc.shape[:2] + (2 - vc.shape[2],) + vc.shape[3:], np.uint64)], axis=2)
    for W in (1, 2):
        val = np.ascontiguousarray(vc[:, :, :W])
        full = cg.map.counter_lub_many(t(d["clock"]), t(d["ec"]), t(val), ctx=ctx, **kw)
        sh = cs.map_counter_lub_many_sharded(t(d["clock"]), t(d["ec"][:, k0:k1]), t(val[:, k0:k1]), k0, K,
                                             ctx=ctx, **kw)
        o[f"vmap_c{W}_k0"] = np.array([k0, k1], np.int64)
        for nm, a, b in (("clock", full.clock, sh.clock), ("ec", full.ec[k0:k1], sh.ec),
                         ("val", full.val[k0:k1], sh.val), ("keep", full.def_keep, sh.def_keep),
                         ("keys", full.def_keys, sh.def_keys), ("flags", full.flags, sh.flags)):
            if a is not None:
                o[f"vmap_c{W}_full_{nm}"], o[f"vmap_c{W}_sh_{nm}"] = a.cpu().numpy().copy(), b.cpu().numpy().copy()
    oc = np.ascontiguousarray(d["ec"])
    ent = np.ascontiguousarray(vc[:, :, :2])
    R = d["clock"].shape[0]
    full = cg.map.orswot_lub_many(t(d["clock"]), t(d["ec"]), t(oc), t(ent),
                                  torch.zeros(R * K + 1, dtype=torch.int64, device=dev), ctx=ctx, **kw)
    sh = cs.map_orswot_lub_many_sharded(t(d["clock"]), t(d["ec"][:, k0:k1]), t(oc[:, k0:k1]), t(ent[:, k0:k1]),
                                        torch.zeros(R * (k1 - k0) + 1, dtype=torch.int64, device=dev), k0, K,
                                        ctx=ctx, **kw)
    o["vmap_o_k0"] = np.array([k0, k1], np.int64)
    for nm, a, b in (("clock", full.clock, sh.clock), ("ec", full.ec[k0:k1], sh.ec), ("oc", full.oc[k0:k1], sh.oc),
                     ("ent", full.ent[k0:k1], sh.ent), ("keep", full.def_keep, sh.def_keep),
                     ("keys", full.def_keys, sh.def_keys), ("flags", full.flags, sh.flags)):
        if a is not None:
            o[f"vmap_o_full_{nm}"], o[f"vmap_o_sh_{nm}"] = a.cpu().numpy().copy(), b.cpu().numpy().copy()
    # Map with device offsets that differ between the ranks (same G and D, so the agreed header
    # matches): the offsets' hash in the flags exchange differs, so BOTH ranks raise EINVAL
    if Dn >= 2:
        c2 = np.stack([d["clock"], d["clock"]])
        e2 = np.stack([d["ec"], d["ec"]])
        v2 = np.stack([d["vclk"], d["vclk"]])
        w2 = np.stack([d["vval"], d["vval"]])
        k0, k1 = cdist.shard_range(K, rank, world)
        split = 1 if rank == 0 else 2
        offd = torch.tensor([0, split, Dn], dtype=torch.int64, device=dev)
        try:
            cs.map_lub_many_sharded(t(c2), t(e2[:, :, k0:k1]), t(v2[:, :, k0:k1]), t(w2[:, :, k0:k1]), k0, K,
                                    def_off=offd, def_row=kw["def_row"], def_clock=kw["def_clock"],
                                    def_keys=kw["def_keys"], vout=D.MAP_VOUT, ctx=ctx)
            o["cabi_mapoff_code"] = np.array([0], np.int64)
        except CrdtGpuError as e:
            o["cabi_mapoff_code"] = np.array([e.code], np.int64)
    # Map: only rank 1's key folds to more values than vout=8 (its fold state overflows first, so the
    # C call reruns every rank with the larger state); the flags are global, so BOTH ranks raise the
    # capacity error, then both succeed with vout=16
    d = D.map_overflow_input()
    K = d["ec"].shape[1]
    k0, k1 = (0, K - 1) if rank == 0 else (K - 1, K)
    args = (t(d["clock"][None]), t(d["ec"][None, :, k0:k1]), t(d["vclk"][None, :, k0:k1]),
            t(d["vval"][None, :, k0:k1]), k0, K)
    try:
        cs.map_lub_many_sharded(*args, vout=8, ctx=ctx)
        o["cabi_mapovf_raised"] = np.array([0], np.int64)
    except cg.map.MapCapacityError:
        o["cabi_mapovf_raised"] = np.array([1], np.int64)
    mres = cs.map_lub_many_sharded(*args, vout=D.MAP_OVF_VOUT, ctx=ctx)
    o["cabi_mapovf_k0"] = np.array([k0, k1], np.int64)
    o["cabi_mapovf_ec"], o["cabi_mapovf_vclk"], o["cabi_mapovf_vval"] = h(mres.ec), h(mres.vclk), h(mres.vval)
    o["cabi_mapovf_nval"] = mres.nval.cpu().numpy().copy()
    o["cabi_mapovf_flags"] = mres.flags.cpu().numpy().copy()
    # ranks passing different starting fold states (Vstate 16 vs 0) with an overflowing key: the
    # retry branches on it, so it is part of the agreed call and BOTH ranks get EINVAL
    try:
        cs.map_lub_many_sharded(*args, vout=D.MAP_OVF_VOUT, ctx=ctx, vstate=16 if rank == 0 else 0)
        o["cabi_mapvstate_code"] = np.array([0], np.int64)
    except CrdtGpuError as e:
        o["cabi_mapvstate_code"] = np.array([e.code], np.int64)
    # a bad argument on ONE rank, none blocks:
    #  * on a plan the ranks agreed earlier (the vclock (G, W) above; the agreed-plan path runs no header
    #    exchange): rank 1's NULL output travels in the check words, the call returns its own error on
    #    rank 1 only, and EVERY rank reports ECOMM at its next sharded call, which runs no collective;
    #  * on plans forgotten after that error (the header exchange): both ranks err in the same call;
    #  * with shagree=1 (the exchange on every call): both ranks err in the call itself.
    # Then good calls work again: the first agrees the plan, the next two take the agreed-plan path.
    x = t(D.lattice_input("vclock")[0])
    outb = torch.empty(x.shape[1], dtype=torch.int64, device=dev)
    o["cabi_pre_errors"] = h(cs.lub_many_sharded("vclock", x, ctx=ctx))  # agrees the plan (G = 1, this W)

    def bad_call(bad):
        try:
            if bad == "null_out":
                ctx.call("crdt_vclock_lub_many_sharded", x.data_ptr(), 1, x.shape[0], x.shape[1], x.shape[1],
                         0, None if rank == 1 else outb.data_ptr())
            else:
                W = x.shape[1] if rank == 0 else x.shape[1] - 2
                ctx.call("crdt_vclock_lub_many_sharded", x.data_ptr(), 1, x.shape[0], W, x.shape[1], 0, outb.data_ptr())
            return 0
        except CrdtGpuError as e:
            return e.code

    o["cabi_error_codes"] = np.array([bad_call("null_out"), bad_call("dims"), bad_call("dims")], np.int64)
    ctx.tune("shagree=1")
    o["cabi_error_codes_sync"] = np.array([bad_call("null_out"), bad_call("dims")], np.int64)
    ctx.tune("shagree=0")
    ctx.timing_reset()
    ctx.set_timing(True)
    o["cabi_after_errors"] = h(cs.lub_many_sharded("vclock", x, ctx=ctx))
    o["cabi_after_errors_cached"] = np.stack([h(cs.lub_many_sharded("vclock", x, ctx=ctx)) for _ in range(2)])
    ctx.synchronize()  # (verifies the last agreed-plan call's check words)
    ctx.set_timing(False)
    o["cabi_agree_calls"] = np.array([ctx.timing("shard_agree")[1], ctx.timing("shard_exchange")[1]], np.int64)
    # config 5 at full per-GPU size: rank k holds replicas [k*R, (k+1)*R) of the
    # 1,048,576-per-rank x 1,024-actor VClock input (bench.py --workload c5's shard), lub through
    # crdt_vclock_lub_many_sharded; the parent checks sampled actor columns against the oracle's fold
    # of all 2M replicas and every column against the max of the ranks' local torch maxima
    R5, A5 = D.C5_R, D.C5_A
    x5 = torch.empty((R5, A5), dtype=torch.int64, device=dev)
    cg.synth_fill(ctx, x5, D.C5_SEED, 0, first_row=rank * R5)
    ctx.timing_reset()
    ctx.set_timing(True)
    o["cabi_c5"] = h(cs.lub_many_sharded("vclock", x5, ctx=ctx))
    ctx.set_timing(False)
    o["cabi_c5_timing_ms"] = np.array([ctx.timing("lub_stream")[0], ctx.timing("shard_exchange")[0],
                                       ctx.timing("shard_agree")[0]], np.float64)
    sign = torch.tensor(-(2**63), dtype=torch.int64, device=dev)
    o["cabi_c5_local_max"] = h((x5 ^ sign).amax(0) ^ sign)
    del x5
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    cs.comm_destroy(ctx)
    return o


if __name__ == "__main__":
    main()
