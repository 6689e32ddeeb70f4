"""Map<K, Map<K2, MVReg<u64>>> lub_many (crdt_map_nested_lub_many, round 5) on one MI355X: the
reference's test type folded at scale.  Op-replay replicas from the oracle's generator (inner writes
and removes read at replicas that have seen more, so removes defer at both levels), tiled to R
replicas, folded in one launch (G = 1); HIP-event kernel time over --reps; parity of the whole fold
against the oracle's left fold (Map::merge restated).  One JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-crdt_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import crdts_gpu as cg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--distinct", type=int, default=256, help="distinct op-replay replicas")
ap.add_argument("--tile", type=int, default=16, help="R = distinct x tile")
ap.add_argument("--keys", type=int, default=64)
ap.add_argument("--inner-keys", type=int, default=8)
ap.add_argument("--actors", type=int, default=8)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
K, K2, A = args.keys, args.inner_keys, args.actors

import oracle as O  # noqa: E402  (input generator and checker only)
from gpu_util import to_dev, to_host  # noqa: E402
from test_gpu_map_nested import canon  # noqa: E402

t0 = time.perf_counter()
maps = O.nested_map_objects(args.distinct, K, K2, A, seed=77, steps=6 * args.distinct, p_irm=0.4, p_ooo=0.7,
                            p_rm=0.2)
maps = maps * args.tile
R = len(maps)
V = max([len(ie.val.vals) for m in maps for e in m.entries.values() for ie in e.val.entries.values()] + [1])
d = O.nested_map_to_dense(maps, K, K2, A, V)
gen_s = time.perf_counter() - t0
torch.cuda.set_device(0)
ctx = cg.Context(0)
D = d["def_row"].shape[0]
kw = dict(def_off=[0, D], def_row=torch.from_numpy(d["def_row"].astype(np.int32)).cuda(),
          def_clock=to_dev(d["def_clock"]), def_keys=to_dev(d["def_keys"])) if D else {}
Di = d["id_clock"].shape[0]
ikw = dict(id_clock=to_dev(d["id_clock"]), id_keys=to_dev(d["id_keys"])) if Di else {}
args_dev = [to_dev(d[x]) for x in ("clock", "ec", "ic", "iec", "ivc", "ivv")] + [to_dev(d["id_off"])]
res = cg.map.nested_lub_many(*args_dev, ctx=ctx, **ikw, **kw)
torch.cuda.synchronize()
ctx.timing_reset()
ctx.set_timing(True)
for _ in range(args.reps):
    res = cg.map.nested_lub_many(*args_dev, ctx=ctx, **ikw, **kw)
torch.cuda.synchronize()
ctx.set_timing(False)
timings = {nm: ctx.timing(nm) for nm in ("map_nested_fold", "map_nested")}
name, (ms, n) = max(((k, v) for k, v in timings.items() if v[1]), key=lambda kv: kv[1][0], default=("", (0.0, 0)))
t = ms / max(n, 1)
in_bytes = sum(x.numel() * 8 for x in args_dev[:6])
t1 = time.perf_counter()
exp = O.map_fold_objects(maps)
cpu_s = time.perf_counter() - t1
dset = []
if D:
    dset = [(np.array(rm, np.uint64), ks) for rm, ks in cg.map.deferred_set(kw["def_clock"], res.def_keep, res.def_keys)]
idn = res.id_n.cpu().numpy()
idc, idk = to_host(res.id_clock), to_host(res.id_keys)
idef = {k: [(idc[k, i], O.bitmap_members(idk[k, i:i + 1])) for i in range(int(idn[k]))] for k in range(K)}
got = O.dense_to_nested_map(to_host(res.clock), to_host(res.ec), to_host(res.ic), to_host(res.iec),
                            to_host(res.ivc), to_host(res.ivv), res.nval.cpu().numpy(), idef, dset)
print(json.dumps({"op": "map_nested_lub_many", "replicas": R, "distinct_replicas": args.distinct, "keys": K,
                  "inner_keys": K2, "actors": A, "V": V, "outer_deferred": D, "inner_deferred": Di,
                  "timer": name, "kernel_ms": t, "replica_merges_per_s": R / (t / 1e3) if t else None,
                  "input_GBs": in_bytes / (t / 1e3) / 1e9 if t else None,
                  "parity": "ok" if canon(got) == canon(exp) else "MISMATCH",
                  "cpu_baseline": {"replica_merges_per_s": R / cpu_s, "cores": 1, "kind": "port",
                                   "sample": f"the whole fold, oracle Map.merge objects (pure Python), {cpu_s:.1f} s"},
                  "gen_s": gen_s}), flush=True)
