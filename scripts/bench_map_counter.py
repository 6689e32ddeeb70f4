"""Map<u32, GCounter> (W = 1) and Map<u32, PNCounter> (W = 2) lub_many at config-4 scale (16,384
replicas x 1,024 keys x 32 actors, deferred removes) on one MI355X (crdt_map_counter_lub_many).
Inputs: the config-4 generator's replicas (crdts_gpu.synth.map_replicas) with the value rows taken
from its MVReg value clocks (slot 0 = the GCounter / P row, slot 1 = N): well-formed counter rows
bounded by the replica clocks.  HIP-event kernel time, algorithmic bytes (every input row read
once), parity of the GPU fold restricted to a key sample against the oracle's left fold of the
same replicas restricted to those keys (keys are independent given the clocks and the deferred
list), on the first --parity-replicas replicas.  One JSON line per W."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-crdt_amd"), os.path.join(ROOT, "oracle")]
import crdts_gpu as cg  # noqa: E402
from crdts_gpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=16384)
ap.add_argument("--keys", type=int, default=1024)
ap.add_argument("--actors", type=int, default=32)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--sample-keys", type=int, default=6)
ap.add_argument("--parity-replicas", type=int, default=512)
ap.add_argument("--p-def", type=float, default=0.1)  # share of replicas holding deferred removes
args = ap.parse_args()
R, K, A = args.replicas, args.keys, args.actors
torch.cuda.set_device(0)
ctx = cg.Context(0)
inp = synth.map_replicas(ctx, R, K, A, 2, 0x5EED0004, kmax=256, p_def=args.p_def)
D = inp.def_clock.shape[0]
Kw = (K + 63) // 64
u64 = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731

import oracle as O  # noqa: E402  (checker only)

for W in (1, 2):
    val = inp.vclk[:, :, :W].contiguous()  # (R, K, W, A)
    kw = dict(def_off=inp.def_off, def_row=inp.def_row, def_clock=inp.def_clock, def_keys=inp.def_keys) if D else {}
    res = cg.map.counter_lub_many(inp.clock, inp.ec, val, ctx=ctx, **kw)
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    for _ in range(args.steps):
        res = cg.map.counter_lub_many(inp.clock, inp.ec, val, ctx=ctx, check=False, **kw)
    torch.cuda.synchronize()
    ctx.set_timing(False)
    ms, n = ctx.timing("map_counter_fold")
    kern = ms / n
    alg = R * (A + K * A * (1 + W)) * 8 + D * (A + Kw + 1) * 8 + K * A * (1 + W) * 8 + A * 8
    # parity: the first P replicas, a key sample, against the oracle's left fold of those replicas
    P = min(args.parity_replicas, R)
    rng = np.random.default_rng(W)
    keys = sorted(rng.choice(K, size=min(args.sample_keys, K), replace=False).tolist())
    rows = inp.def_row.cpu().numpy().astype(np.int64)
    Dp = int(np.searchsorted(rows, P))
    kwp = dict(def_off=[0, Dp], def_row=inp.def_row[:Dp].contiguous(), def_clock=inp.def_clock[:Dp].contiguous(),
               def_keys=inp.def_keys[:Dp].contiguous()) if Dp else {}
    sub = cg.map.counter_lub_many(inp.clock[:P].contiguous(), inp.ec[:P].contiguous(), val[:P].contiguous(),
                                  ctx=ctx, **kwp)
    hc, he, hv = u64(inp.clock[:P]), u64(inp.ec[:P]), u64(val[:P])
    dcl, dks = u64(inp.def_clock[:Dp]) if Dp else None, u64(inp.def_keys[:Dp]) if Dp else None
    ks = np.array(keys)
    t0 = time.perf_counter()
    maps = []
    for r in range(P):
        deferred = []
        for d in range(Dp):
            if rows[d] == r:
                named = {i for i, k in enumerate(keys) if (int(dks[d][k // 64]) >> (k % 64)) & 1}
                if named:
                    deferred.append((dcl[d], named))
        maps.append(O.dense_to_map_counter(hc[r], he[r][ks], hv[r][ks], deferred))
    exp = O.map_fold_objects(maps)
    cpu_s = time.perf_counter() - t0
    gc, ge, gv = u64(sub.clock), u64(sub.ec)[ks], u64(sub.val)[ks]
    got = O.dense_to_map_counter(gc, ge, gv)
    ok = got.clock == exp.clock and got.entries == exp.entries
    print(json.dumps({
        "op": "map_counter_lub_many", "value": "GCounter" if W == 1 else "PNCounter", "replicas": R, "keys": K,
        "actors": A, "W": W, "deferred": D, "kernel_ms": kern, "algorithmic_bytes": alg,
        "kernel_GBs": alg / kern / 1e6, "frac_of_8TBs": alg / kern / 8e9, "replica_merges_per_s": R / kern * 1e3,
        "parity": "ok" if ok else "MISMATCH", "parity_sample": f"first {P} replicas, keys {keys}",
        "cpu_baseline": {"replica_merges_per_s": P / cpu_s, "cores": 1, "kind": "port",
                         "sample": f"oracle Map.merge fold of {P} replicas restricted to {len(keys)} keys "
                                   f"(pure Python objects; not comparable per byte)"},
    }), flush=True)
