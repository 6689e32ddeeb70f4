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
    out["lib"] = np.frombuffer(cg._abi.LIB_PATH.encode(), np.uint8)
    torch.cuda.synchronize()
    np.savez(os.path.join(args.out, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
