"""Batched Map<K, MVReg<u64>> CmRDT::apply on one MI355X: N states x T ops each
(crdt_map_apply_batch), device-generated streams (crdts_gpu.synth.map_op_streams: 80% writes of a
random key with a new dot, 20% single-key removes, a third of them from the future so they defer).
States are reset before every rep (a second pass over a stream would see every dot).  HIP-event
kernel time; parity of a state sample against the oracle's Map.apply (reference-shaped objects);
CPU baseline = that oracle (pure Python, one thread) on the sample.  One JSON line."""
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
ap.add_argument("--states", type=int, default=65536)
ap.add_argument("--ops", type=int, default=64)
ap.add_argument("--keys", type=int, default=256)
ap.add_argument("--actors", type=int, default=32)
ap.add_argument("--vals", type=int, default=4)
ap.add_argument("--dcap", type=int, default=16)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--tune", default="")
ap.add_argument("--contig", action="store_true", help="the states in one contiguous device block")
args = ap.parse_args()
N, T, K, A, V, Dcap = args.states, args.ops, args.keys, args.actors, args.vals, args.dcap
Kw = (K + 63) // 64

torch.cuda.set_device(0)
ctx = cg.Context(0)
if args.tune:
    ctx.tune(args.tune)
ops = cg.synth.map_op_streams(N, T, K, A, seed=0x5EED000A, device="cuda")
shapes = ((N, A), (N, K, A), (N, K, V, A), (N, K, V), (N, Dcap, A), (N, Dcap, Kw))
block = None
if args.contig:  # the states in one physically contiguous device block (crdt_device_alloc)
    block = ctx.device_empty((sum((int(np.prod(sh)) + 511) // 512 * 512 for sh in shapes),))
if block is not None:
    views, at = [], 0
    for sh in shapes:
        n = int(np.prod(sh))
        views.append(block[at:at + n].view(sh).zero_())
        at += (n + 511) // 512 * 512
    clock, ec, vclk, vval, dcl, dks = views
else:
    clock, ec, vclk, vval, dcl, dks = (torch.zeros(sh, dtype=torch.int64, device="cuda") for sh in shapes)
print(f"# states: {'contiguous block' if block is not None else 'torch allocator'}", file=sys.stderr, flush=True)
cnt = torch.zeros(N, dtype=torch.int32, device="cuda")


def reset():
    for t in (clock, ec, vclk, vval):
        t.zero_()
    cnt.zero_()


def run():
    return cg.map.apply_batch(clock, ec, vclk, vval, dcl, dks, cnt, ops, ctx=ctx)


reset()
run()
torch.cuda.synchronize()
ctx.timing_reset()
for _ in range(args.reps):
    reset()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    status = run()
    torch.cuda.synchronize()
    ctx.set_timing(False)
ms, n = ctx.timing("map_apply")
t = ms / n / 1e3
st = status.cpu().numpy()

import oracle as O  # noqa: E402  (checker and CPU baseline only)

host = {f: getattr(ops, f).cpu().numpy() for f in ops._fields}
sample = np.sort(np.random.default_rng(0).choice(N, size=min(N, 64), replace=False))


def obj_ops(s):
    out = []
    for o in range(int(host["op_off"][s]), int(host["op_off"][s + 1])):
        row = host["clk_pool"][host["clk_row"][o]].view(np.uint64)
        clk = O.VClock({a: int(v) for a, v in enumerate(row) if v})
        k = int(host["keys"][host["key_off"][o]])
        if host["kind"][o] == 0:
            out.append(O.MapUp(O.Dot(int(host["actor"][o]), int(host["counter"][o])), k,
                               O.MVRegPut(clk, int(host["val"][o]))))
        else:
            out.append(O.MapRm(clk, {k}))
    return out


streams = [obj_ops(int(s)) for s in sample]
t0 = time.perf_counter()
exp = []
for ops_s in streams:
    m = O.Map(O.MVReg)
    for op in ops_s:
        m.apply(op)
    exp.append(m)
cpu_s = time.perf_counter() - t0
sidx = torch.from_numpy(sample).cuda()
gc, ge, gv, gw = (x[sidx].cpu().numpy().view(np.uint64) for x in (clock, ec, vclk, vval))
ok = not (st & 1).any() and not (st & 16).any()
for i, m in enumerate(exp):
    g = O.dense_to_map(gc[i], ge[i], gv[i], gw[i])
    ok &= g.clock == m.clock and g.entries == m.entries
    ok &= int(cnt[int(sample[i])].item()) == len(m.deferred)

print(json.dumps({
    "op": "map_apply_batch", "states": N, "ops_per_state": T, "keys": K, "actors": A, "vals": V, "dcap": Dcap,
    "removes": int((host["kind"] == 1).sum()), "deferred_left": int(cnt.sum().item()),
    "overflow_states": int(((st & 17) != 0).sum()), "kernel_us": t * 1e6, "ops_per_s": N * T / t,
    "parity": "ok" if ok else "MISMATCH", "parity_states": int(len(sample)),
    "cpu_baseline": {"ops_per_s": len(sample) * T / cpu_s, "cores": 1, "kind": "port",
                     "sample": f"{len(sample)} states x {T} ops, oracle Map.apply (pure Python objects)"},
}), flush=True)
