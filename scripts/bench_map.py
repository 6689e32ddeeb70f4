"""Map<u32, MVReg<u64>> lub_many at BASELINE config 4 scale (16,384 replicas x 1,024 keys x 32
actors, 2 value slots per key, ~12.3 GiB, deferred removes) on one MI355X: throughput, the HBM
roofline of the fold kernel, parity against the oracle on a key sample (keys are independent
given the replica clocks and deferred list, so the reference fold over every replica restricted
to a key subset must equal the GPU result restricted to it), and the reference fold (the
oracle's C++ restatement over map-based states) timed on a replica subsample as CPU baseline.
Prints one JSON line per measurement."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-crdt_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=16384)
ap.add_argument("--keys", type=int, default=1024)
ap.add_argument("--actors", type=int, default=32)
ap.add_argument("--slots", type=int, default=2)
ap.add_argument("--kmax", type=int, default=256)
ap.add_argument("--p-def", type=float, default=0.1)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--sample-keys", type=int, default=8)
ap.add_argument("--cpu-replicas", type=int, default=4096, help="replica subsample for the CPU fold")
ap.add_argument("--no-parity", action="store_true")
ap.add_argument("--contig", action=argparse.BooleanOptionalAction, default=True,
                help="the replicas in one contiguous device block (as bench.py's c4 block)")
args = ap.parse_args()

R, K, A, V = args.replicas, args.keys, args.actors, args.slots
SEED = 0x5EED0004
T0 = time.time()


def log(msg):
    print(f"[{time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


torch.cuda.set_device(0)
ctx = cg.Context(0)
in_bytes = R * (K * (A * 8 + V * A * 8 + V * 8) + A * 8)
log(f"generating {R}x{K}x{A} V={V} ({in_bytes / 2**30:.2f} GiB)")
t0 = time.time()
inp = synth.map_replicas(ctx, R, K, A, V, SEED, kmax=args.kmax, p_def=args.p_def, contig=args.contig)
torch.cuda.synchronize()
gen_s = time.time() - t0
D = inp.def_clock.shape[0]
Kw = (K + 63) // 64
VOUT = 4
alg_bytes = in_bytes + D * (A + Kw + 1) * 8 + K * (A + VOUT * A + VOUT) * 8 + A * 8
log(f"generated in {gen_s:.1f}s, {D} deferred removes")


def run():
    return cg.map.lub_many(inp.clock, inp.ec, inp.vclk, inp.vval, def_off=inp.def_off,
                           def_row=inp.def_row, def_clock=inp.def_clock, def_keys=inp.def_keys,
                           vout=VOUT, ctx=ctx, check=False)


for _ in range(2):
    res = run()
torch.cuda.synchronize()
ctx.timing_reset()
ctx.set_timing(True)
t1 = time.perf_counter()
for _ in range(args.steps):
    res = run()
torch.cuda.synchronize()
wall = (time.perf_counter() - t1) / args.steps
ms, n = ctx.timing("map_fold")
ctx.set_timing(False)
kern = ms / n / 1e3
flags = res.flags.cpu().numpy()
out = {"workload": f"map<u32,mvreg<u64>> lub {R}x{K}x{A} V={V}", "replicas": R, "keys": K,
       "actors": A, "slots": V, "deferred": D, "wall_ms": wall * 1e3, "kernel_ms": kern * 1e3, "tune": os.environ.get("CRDT_TUNE", ""),
       "algorithmic_bytes": alg_bytes, "kernel_GBs": alg_bytes / kern / 1e9,
       "frac_of_8TBs": alg_bytes / kern / 8e12, "replica_merges_per_s": R / wall,
       "flags": int(np.bitwise_or.reduce(flags)) if flags.size else 0, "input_alloc": inp.alloc}
print(json.dumps(out), flush=True)
if args.no_parity:
    sys.exit(0)

# ---- parity on sampled keys vs the oracle fold (reference semantics) ---------------------------
import oracle as O  # noqa: E402  (checker only)

rng = np.random.default_rng(1)
keys = np.sort(rng.choice(K, size=min(K, args.sample_keys), replace=False))
log(f"parity: regenerating keys {keys.tolist()} on the CPU")
dfr = O.synth_map_deferred(SEED, R, K, A, args.kmax, p_def=args.p_def)
d = O.synth_map(SEED, R, K, A, V, args.kmax, keys=keys, deferred=dfr)
# the device generator must agree with the restatement on these keys
tk = torch.from_numpy(keys).cuda()
for nm in ("clock", "ec", "vclk", "vval"):
    t = getattr(inp, nm)
    h = (t if nm == "clock" else t[:, tk]).cpu().numpy().view(np.uint64)
    assert np.array_equal(h, d[nm]), f"synth {nm} mismatch"
log("parity: oracle fold over all replicas, key sample")
t2 = time.time()
exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], dfr[0], dfr[1],
                 O.restrict_deferred_keys(dfr[2], keys), VOUT)
host = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731
ok = (np.array_equal(host(res.clock), exp[0]) and np.array_equal(host(res.ec)[keys], exp[1])
      and np.array_equal(host(res.vclk)[keys], exp[2]) and np.array_equal(host(res.vval)[keys], exp[3])
      and np.array_equal(res.nval.cpu().numpy()[keys], exp[4]))
got = cg.map.deferred_set(inp.def_clock, res.def_keep, res.def_keys)
pos = {int(k): i for i, k in enumerate(keys)}
got_sub = {(c, frozenset(pos[k] for k in ks if k in pos)) for c, ks in got}
got_sub = {x for x in got_sub if x[1]}
exp_sub = {x for x in exp[5] if x[1]}
ok = ok and got_sub == exp_sub and not out["flags"]
log(f"parity {'ok' if ok else 'MISMATCH'} ({time.time() - t2:.1f}s)")

# ---- CPU baseline: the restated reference fold on a replica subsample, all keys ---------------
Rc = min(R, args.cpu_replicas)
log(f"cpu baseline: reference fold of {Rc} full replicas")
dfc = O.synth_map_deferred(SEED, Rc, K, A, args.kmax, p_def=args.p_def)
dc = O.synth_map(SEED, Rc, K, A, V, args.kmax, deferred=dfc)
res_c = O.map_fold(dc["clock"], dc["ec"], dc["vclk"], dc["vval"], dfc[0], dfc[1], dfc[2], VOUT)
fold_s = res_c[6]
print(json.dumps({"parity": "ok" if ok else "MISMATCH", "sample_keys": keys.tolist(),
                  "surviving_deferred_in_sample": len(exp_sub), "gen_s": gen_s,
                  "cpu_baseline": {"value": Rc / fold_s, "unit": "replica-merges/s", "cores": 1,
                                   "kind": "port",
                                   "sample": f"first {Rc} of the {R} replicas, all {K} keys; left fold "
                                             f"of the restated Map::merge over std::map states "
                                             f"(oracle/ref_fold.cpp), 1 thread, ingest excluded; "
                                             f"{fold_s:.2f} s of fold"}}), flush=True)
sys.exit(0 if ok else 3)
