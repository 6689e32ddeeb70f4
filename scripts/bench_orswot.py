"""Orswot lub_many at BASELINE config 3 scale (65,536 replicas x 4,096 members x 64 actors,
128 GiB of entries, deferred removes) on one MI355X: throughput, HBM roofline of the join
kernel, and parity against the oracle on a sample of members (the merge is independent per
member given the clocks, so the reference fold restricted to a member subset must equal the
GPU result restricted to it — including the surviving deferred removes)."""
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
ap.add_argument("--replicas", type=int, default=65536)
ap.add_argument("--members", type=int, default=4096)
ap.add_argument("--actors", type=int, default=64)
ap.add_argument("--kmax", type=int, default=48)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--sample-members", type=int, default=6)
ap.add_argument("--tune", nargs="*", default=[""])
ap.add_argument("--map-oracle-max", type=int, default=8192,
                help="largest R checked with the map-based oracle fold (slow: O(R x D))")
args = ap.parse_args()

R, M, A = args.replicas, args.members, args.actors
T0 = time.time()


def log(msg):
    print(f"[{time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


torch.cuda.set_device(0)
ctx0 = cg.Context(0)
t0 = time.time()
log(f"generating {R}x{M}x{A} ({R * M * A * 8 / 2**30:.1f} GiB entries)")
inp = synth.orswot_replicas(ctx0, R, M, A, seed=0x5EED0003, kmax=args.kmax, p_def=0.1)
torch.cuda.synchronize()
log("generated")
gen_s = time.time() - t0
D = inp.def_clock.shape[0]
goff = [0, D]
ebytes = R * M * A * 8 + R * A * 8
results = []
res = None
for tune in args.tune:
    os.environ["CRDT_TUNE"] = tune
    ctx = cg.Context(0)
    log(f"tune {tune!r}: warmup")
    for _ in range(2):
        res = cg.orswot.lub_many(inp.clock, inp.entries, def_off=goff, def_clock=inp.def_clock,
                                 def_members=inp.def_members, ctx=ctx)
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        res = cg.orswot.lub_many(inp.clock, inp.entries, def_off=goff, def_clock=inp.def_clock,
                                 def_members=inp.def_members, ctx=ctx)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t1) / args.steps
    ms, n = ctx.timing("orswot_join")
    ctx.set_timing(False)
    kern = ms / n / 1e3
    out = {"tune": tune, "R": R, "M": M, "A": A, "D": D, "wall_ms": wall * 1e3, "join_ms": kern * 1e3,
           "join_GBs": ebytes / kern / 1e9, "join_frac_of_8TBs": ebytes / kern / 8e12,
           "replica_merges_per_s": R / wall}
    results.append(out)
    print(json.dumps(out), flush=True)
    ctx.close()

# ---- parity on sampled members vs the oracle fold (reference semantics) ----------------------
import oracle as O  # noqa: E402  (checker only)

log("parity: copying sampled members")
rng = np.random.default_rng(1)
msub = np.sort(rng.choice(M, size=min(M, args.sample_members), replace=False))
clock_h = inp.clock.cpu().numpy().view(np.uint64)
ent_h = inp.entries[:, torch.from_numpy(msub).cuda(), :].cpu().numpy().view(np.uint64)
dcl_h = inp.def_clock.cpu().numpy().view(np.uint64)
dmem_h = inp.def_members.cpu().numpy().view(np.uint64)
Ms = len(msub)
Mws = (Ms + 63) // 64
sub_mem = np.zeros((D, Mws), dtype=np.uint64)
for j, m in enumerate(msub):
    bit = (dmem_h[:, m // 64] >> np.uint64(m % 64)) & np.uint64(1)
    sub_mem[:, j // 64] |= bit << np.uint64(j % 64)
# the generator's replicas, regenerated on the CPU for a few rows, must match HBM
rows = rng.choice(R, size=3, replace=False)
for r in rows:
    c_cpu, e_cpu = O.synth_orswot(0x5EED0003, 1, M, A, args.kmax, row0=int(r))
    dr = np.nonzero(np.repeat(np.arange(R), np.diff(inp.def_off.astype(np.int64))) == r)[0]
    e_cpu = O.apply_rm_rows(e_cpu, [0] * len(dr), dcl_h[dr], dmem_h[dr])
    assert np.array_equal(c_cpu[0], clock_h[r]), "synth clock mismatch"
    assert np.array_equal(e_cpu[0][msub], ent_h[r]), "synth entries mismatch"
t2 = time.time()
if R <= args.map_oracle_max:
    log("parity: oracle fold (map-based reference restatement)")
    oc, oe, odef, fold_s = O.orswot_fold(clock_h, ent_h, inp.def_off, dcl_h, sub_mem)
    oracle_kind = "orswot_fold (std::unordered_map states, oracle/ref_fold.cpp)"
else:
    # The map-based restatement re-applies every surviving deferred remove on every merge, as
    # the reference does (orswot.rs:141-147): O(R x D) — minutes at config-3 size.  Its dense
    # equivalent (join fold, then each remove once), cross-checked against it in
    # tests/test_oracle_twins.py, checks the full-size result.
    log("parity: dense oracle fold (join fold + removes, equivalent to the map-based fold)")
    t_f = time.time()
    oc, oe, odef = O.dense_orswot_lub(clock_h, ent_h, dcl_h, sub_mem)
    fold_s = time.time() - t_f
    oracle_kind = "dense_orswot_lub (numpy, = orswot_fold on every tested input)"
got_c = res.clock.cpu().numpy().view(np.uint64)
got_e = res.entries[torch.from_numpy(msub).cuda()].cpu().numpy().view(np.uint64)
keep = res.def_keep.cpu().numpy()
gmem = res.def_members.cpu().numpy().view(np.uint64)
got_def = set()
for d in np.nonzero(keep)[0]:
    ms = frozenset(j for j, m in enumerate(msub.tolist()) if (int(gmem[d, m // 64]) >> (m % 64)) & 1)
    got_def.add((tuple(int(x) for x in dcl_h[d]), ms))
ok = np.array_equal(oc, got_c) and np.array_equal(oe, got_e) and got_def == odef
print(json.dumps({"parity": "ok" if ok else "MISMATCH", "oracle": oracle_kind, "sample_members": msub.tolist(),
                  "surviving_deferred": len(odef), "oracle_fold_s": fold_s, "gen_s": gen_s,
                  "check_s": time.time() - t2}), flush=True)
sys.exit(0 if ok else 3)
