"""Batched Orswot CmRDT::apply on one MI355X: N states x T ops each (crdt_orswot_apply_batch),
device-generated streams (crdts_gpu.synth.orswot_op_streams: 80% single-member adds with new
dots, 20% single-member removes, 30% of them from the future so they defer).  States are reset
before every rep (apply is not idempotent over a stream: a second pass would see every dot).
HIP-event kernel time; parity of a state sample against the C++ twin (oracle, std containers);
CPU baseline = the same twin on a bounded sample of states, one thread.  One JSON line."""
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
ap.add_argument("--members", type=int, default=1024)
ap.add_argument("--actors", type=int, default=64)
ap.add_argument("--dcap", type=int, default=16)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--tune", default="")
ap.add_argument("--p-rm", type=float, default=0.2)
ap.add_argument("--p-future", type=float, default=0.3)
ap.add_argument("--contig", action="store_true", help="the states in one contiguous device block")
ap.add_argument("--cpu-s", type=float, default=10.0, help="CPU-baseline budget (0: none)")
args = ap.parse_args()
N, T, M, A, Dcap = args.states, args.ops, args.members, args.actors, args.dcap
Mw = (M + 63) // 64

torch.cuda.set_device(0)
ctx = cg.Context(0)
if args.tune:
    ctx.tune(args.tune)
t0 = time.time()
ops = cg.synth.orswot_op_streams(N, T, M, A, seed=0x5EED0009, p_rm=args.p_rm, p_future=args.p_future, device="cuda")
shapes = ((N, A), (N, M, A), (N, Dcap, A), (N, Dcap, Mw))
block = None
if args.contig:  # the states in one physically contiguous device block (crdt_device_alloc)
    pad = lambda n: (n + 511) // 512 * 512  # noqa: E731
    block = ctx.device_empty((sum(pad(int(np.prod(sh))) for sh in shapes),))
if block is not None:
    views, at = [], 0
    for sh in shapes:
        n = int(np.prod(sh))
        views.append(block[at:at + n].view(sh).zero_())
        at += (n + 511) // 512 * 512
    clock, entries, dcl, dmb = views
else:
    clock, entries, dcl, dmb = (torch.zeros(sh, dtype=torch.int64, device="cuda") for sh in shapes)
print(f"# states: {'contiguous block' if block is not None else 'torch allocator'}", file=sys.stderr, flush=True)
cnt = torch.zeros(N, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
print(f"# generated {N * T} ops in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)


def reset():
    clock.zero_()
    entries.zero_()
    cnt.zero_()


reset()
status = cg.orswot.apply_batch(clock, entries, dcl, dmb, cnt, ops, ctx=ctx)  # warm-up
torch.cuda.synchronize()
ctx.timing_reset()
for _ in range(args.reps):
    reset()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    status = cg.orswot.apply_batch(clock, entries, dcl, dmb, cnt, ops, ctx=ctx)
    torch.cuda.synchronize()
    ctx.set_timing(False)
ms, n = ctx.timing("orswot_apply")
t = ms / n / 1e3
st = status.cpu().numpy()
n_rm = int((ops.kind == 1).sum().item())
n_add = N * T - n_rm
# minimal HBM traffic: op headers (kind 1 + actor 4 + counter 8 + rm_row 4 + member 4 +
# mem_off 8 + op_off) + per add one entry cell read+write + per rm its clock row and one member
# row read (+ write back, counted once) + per state its clock read+write
op_bytes = N * T * (1 + 4 + 8 + 4 + 4 + 8) + 8 * (N + 1)
traffic = op_bytes + n_add * 16 + n_rm * (8 * A + 16 * A) + N * 16 * A

# parity: every state of a sample, against the C++ twin
import oracle as O  # noqa: E402  (checker and CPU baseline only)

rng = np.random.default_rng(0)
sample = np.sort(rng.choice(N, size=min(N, 256), replace=False))
host = [x.cpu().numpy() for x in ops]


def sub(states):
    ob = host[0]
    o_idx = np.concatenate([np.arange(ob[s], ob[s + 1]) for s in states])
    off = np.concatenate([[0], np.cumsum([ob[s + 1] - ob[s] for s in states])]).astype(np.uint64)
    mo = host[6]
    m_idx = np.concatenate([np.arange(mo[o], mo[o + 1]) for o in o_idx])
    moff = np.concatenate([[0], np.cumsum(mo[o_idx + 1] - mo[o_idx])]).astype(np.uint64)
    return (off, host[1][o_idx], host[2][o_idx], host[3][o_idx], np.arange(len(o_idx), dtype=np.uint32),
            host[5][host[4][o_idx]], moff, host[7][m_idx])


oc, oe, ond, _ = O.orswot_apply_streams(len(sample), M, A, *sub(sample))
sidx = torch.from_numpy(sample).cuda()
gc = clock[sidx].cpu().numpy().view(np.uint64)
ge = entries[sidx].cpu().numpy().view(np.uint64)
gn = cnt[sidx].cpu().numpy()
ok = (np.array_equal(gc, oc) and np.array_equal(ge, oe) and np.array_equal(gn, ond.astype(np.int32))
      and not (st & 1).any())

# CPU baseline: the twin on a bounded sample of states (~10 s), one thread
cpu_states, cpu_s, k = 0, 0.0, 0
while cpu_s < args.cpu_s and k * 4096 < N:
    blk = np.arange(k * 4096, min(N, (k + 1) * 4096))
    _, _, _, secs = O.orswot_apply_streams(len(blk), M, A, *sub(blk))
    cpu_states += len(blk)
    cpu_s += secs
    k += 1

print(json.dumps({
    "op": "orswot_apply_batch", "states": N, "ops_per_state": T, "members": M, "actors": A, "dcap": Dcap,
    "adds": n_add, "removes": n_rm, "deferred_left": int(cnt.sum().item()), "overflow_states": int((st & 1).astype(bool).sum()),
    "kernel_us": t * 1e6, "ops_per_s": N * T / t, "min_traffic_GBs": traffic / t / 1e9,
    "parity": "ok" if ok else "MISMATCH", "parity_states": int(len(sample)),
    "p_rm": args.p_rm, "p_future": args.p_future,
    "cpu_baseline": None if not cpu_states else {"ops_per_s": cpu_states * T / cpu_s, "cores": 1, "kind": "port",
                     "sample": f"{cpu_states} states x {T} ops, C++ twin over std containers, {cpu_s:.2f} s"},
}), flush=True)
