"""Map<u32, Orswot<u32>> lub_many (crdt_map_orswot_lub_many) at config-4 scale: 16,384 replicas x
1,024 keys x 32 actors, M = 4 members per nested set, on one MI355X.  Inputs (synthetic, generated
in HBM by torch): replica clocks, for each key present with probability 1/2 an entry clock and a
nested Orswot clock drawn under the replica clock, member dots under the nested clock (a member
present with probability 1/2); no deferred removes at either level (the fold is exact for any input;
the removes' own paths are covered by tests/test_gpu_map_orswot.py).  --input causal instead takes
the config-4 generator's replicas (causally closed states of one op history, crdts_gpu.synth
.map_replicas, no Map-level removes; key k written by actors k % A and (k+1) % A): the entry clock as
the nested Orswot clock, writer i's live dot on k as the dot of member i (i = 0, 1: a member keeps
its writer across replicas), members 2.. absent.  HIP-event kernel time,
algorithmic bytes (every input row read once), parity of the GPU fold of the first
--parity-replicas replicas against the oracle's left fold restricted to a key sample."""
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

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=16384)
ap.add_argument("--keys", type=int, default=1024)
ap.add_argument("--actors", type=int, default=32)
ap.add_argument("--members", type=int, default=4)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--sample-keys", type=int, default=4)
ap.add_argument("--parity-replicas", type=int, default=256)
ap.add_argument("--input", choices=("random", "causal"), default="random")
ap.add_argument("--contig", action="store_true", help="the replicas in one contiguous device block")
ap.add_argument("--split-probe", type=int, default=0,
                help="also time the fold of the replicas cut into P groups (level 1 of a replica split)")
args = ap.parse_args()
R, K, A, M = args.replicas, args.keys, args.actors, args.members
torch.cuda.set_device(0)
ctx = cg.Context(0)
gen = torch.Generator(device="cuda").manual_seed(0x5EED0004)
dev = torch.device("cuda", 0)


def below(hi):  # a random row under hi (per element in [0, hi]), 0 with probability 1/2
    x = (torch.rand(hi.shape, generator=gen, device=dev) * (hi.double() + 1)).long()
    return x * (torch.rand(hi.shape, generator=gen, device=dev) < 0.5)


if args.input == "random":
    clock = torch.randint(1, 1 << 20, (R, A), generator=gen, device=dev)
    pres = (torch.rand((R, K, 1), generator=gen, device=dev) < 0.5)
    ec = below(clock[:, None, :].expand(R, K, A)) * pres
    ec[..., 0] += pres[..., 0].long() * (ec.sum(-1) == 0)  # a present key has a non-empty entry clock
    oc = below(clock[:, None, :].expand(R, K, A)) * pres
    ent = torch.empty((R, K, M, A), dtype=torch.int64, device=dev)
    for m in range(M):
        ent[:, :, m] = below(oc) * (torch.rand((R, K, 1), generator=gen, device=dev) < 0.5)
else:
    from crdts_gpu import synth  # noqa: E402
    inp = synth.map_replicas(ctx, R, K, A, 2, 0x5EED0004, kmax=256, p_def=0.0)
    clock, ec = inp.clock, inp.ec
    oc = ec.clone()
    ent = torch.zeros((R, K, M, A), dtype=torch.int64, device=dev)
    act = torch.arange(A, device=dev)
    for i in range(min(M, 2)):  # member i: writer (k + i) % A's dot
        ent[:, :, i] = ec * (act[None, :] == (torch.arange(K, device=dev)[:, None] + i) % A)[None]
    del inp
if args.contig:  # the replica arrays moved into one physically contiguous device block (crdt_device_alloc)
    arrs = [clock, ec, oc, ent]
    pad = lambda n: (n + 511) // 512 * 512  # noqa: E731
    block = ctx.device_empty((sum(pad(t.numel()) for t in arrs),))
    if block is not None:
        views, at = [], 0
        for t in arrs:
            v = block[at:at + t.numel()].view(t.shape)
            v.copy_(t)
            views.append(v)
            at += pad(t.numel())
        clock, ec, oc, ent = views
        del arrs, t
        torch.cuda.empty_cache()
vd_off = torch.zeros(R * K + 1, dtype=torch.int64, device=dev)
torch.cuda.synchronize()

res = cg.map.orswot_lub_many(clock, ec, oc, ent, vd_off, ctx=ctx)
torch.cuda.synchronize()
ctx.timing_reset()
ctx.set_timing(True)
for _ in range(args.steps):
    res = cg.map.orswot_lub_many(clock, ec, oc, ent, vd_off, ctx=ctx, check=False)
torch.cuda.synchronize()
ctx.set_timing(False)
ms, n = ctx.timing("map_orswot_fold")
kern = ms / n
alg = R * (A + K * A * (2 + M)) * 8 + K * A * (2 + M) * 8 + A * 8
if args.split_probe > 1:
    Ps = args.split_probe
    v = lambda t: t.view((Ps, R // Ps) + tuple(t.shape[1:]))  # noqa: E731
    for _ in range(2):
        cg.map.orswot_lub_many(v(clock), v(ec), v(oc), v(ent), vd_off, ctx=ctx, check=False)
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    for _ in range(args.steps):
        cg.map.orswot_lub_many(v(clock), v(ec), v(oc), v(ent), vd_off, ctx=ctx, check=False)
    torch.cuda.synchronize()
    ctx.set_timing(False)
    ms1, n1 = ctx.timing("map_orswot_fold")
    print(json.dumps({"split_probe": Ps, "level1_kernel_ms": ms1 / n1, "whole_kernel_ms": kern}), flush=True)

import oracle as O  # noqa: E402  (checker only)

P = min(args.parity_replicas, R)
rng = np.random.default_rng(4)
keys = sorted(rng.choice(K, size=min(args.sample_keys, K), replace=False).tolist())
ks = torch.tensor(keys, device=dev)
sub = cg.map.orswot_lub_many(clock[:P].contiguous(), ec[:P, ks].contiguous(), oc[:P, ks].contiguous(),
                             ent[:P, ks].contiguous(), torch.zeros(P * len(keys) + 1, dtype=torch.int64, device=dev),
                             ctx=ctx)
u64 = lambda t: t.cpu().numpy().view(np.uint64)  # noqa: E731
hc, he, ho, hm = u64(clock[:P]), u64(ec[:P, ks]), u64(oc[:P, ks]), u64(ent[:P, ks])
t0 = time.perf_counter()
maps = [O.dense_to_map_orswot(hc[r], he[r], ho[r], hm[r]) for r in range(P)]
exp = O.map_fold_objects(maps)
cpu_s = time.perf_counter() - t0
got = O.dense_to_map_orswot(u64(sub.clock), u64(sub.ec), u64(sub.oc), u64(sub.ent))
# and the full launch restricted to the same keys (the keys are independent: same fold, same result)
full_sub = cg.map.orswot_lub_many(clock[:P].contiguous(), ec[:P].contiguous(), oc[:P].contiguous(),
                                  ent[:P].contiguous(), torch.zeros(P * K + 1, dtype=torch.int64, device=dev), ctx=ctx)
ok = (got.clock == exp.clock and got.entries == exp.entries
      and np.array_equal(u64(full_sub.ec)[keys], u64(sub.ec)) and np.array_equal(u64(full_sub.ent)[keys], u64(sub.ent)))
print(json.dumps({
    "op": "map_orswot_lub_many", "input": args.input, "replicas": R, "keys": K, "actors": A, "members": M, "kernel_ms": kern,
    "algorithmic_bytes": alg, "kernel_GBs": alg / kern / 1e6, "frac_of_8TBs": alg / kern / 8e9,
    "replica_merges_per_s": R / kern * 1e3, "parity": "ok" if ok else "MISMATCH",
    "parity_sample": f"first {P} replicas, keys {keys}",
    "cpu_baseline": {"replica_merges_per_s": P / cpu_s, "cores": 1, "kind": "port",
                     "sample": f"oracle Map.merge fold of {P} replicas restricted to {len(keys)} keys "
                               f"(pure Python objects; not comparable per byte)"},
}), flush=True)
