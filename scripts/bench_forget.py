"""Batched Causal::forget of whole states on one MI355X: Orswot 16,384 states x 4,096 members x
64 actors (32 GiB of entry clocks) and Map<K, MVReg> 16,384 x 1,024 keys x 32 actors x V=2,
every state forgetting its own random clock.  HIP-event kernel time of the dominant launch vs
the algorithmic bytes (read + write of every entry row); parity of a state sample against the
dense rule (keep x iff x > y).  One JSON line per type."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-crdt_amd")]
import crdts_gpu as cg  # noqa: E402

torch.cuda.set_device(0)
ctx = cg.Context(0)


def timed(name, fn, reset, reps=5):
    reset()
    fn()
    torch.cuda.synchronize()
    ctx.timing_reset()
    for _ in range(reps):
        reset()
        torch.cuda.synchronize()
        ctx.set_timing(True)
        fn()
        torch.cuda.synchronize()
        ctx.set_timing(False)
    ms, n = ctx.timing(name)
    return ms / n / 1e3


MAP_ONLY = os.environ.get("FORGET_MAP_ONLY") == "1"  # spread diagnosis: skip the Orswot part
# ---- Orswot
N, M, A = 16384, 4096, 64
src = torch.empty((N if not MAP_ONLY else 1, M, A), dtype=torch.int64, device="cuda")
N = src.shape[0]
cg.synth_fill(ctx, src.view(N * M, A), 0x5EED0021, 0)
src.remainder_(64)  # small counters so the forget clears a fair share
ent = torch.empty_like(src)
clock = torch.empty((N, A), dtype=torch.int64, device="cuda")
cg.synth_fill(ctx, clock, 0x5EED0022, 0)
clock.remainder_(64)
clock0 = clock.clone()
y = torch.empty((N, A), dtype=torch.int64, device="cuda")
cg.synth_fill(ctx, y, 0x5EED0023, 0)
y.remainder_(48)


def reset_o():
    ent.copy_(src)
    clock.copy_(clock0)


t = timed("forget_rows", lambda: cg.orswot.forget_batch(clock, ent, y, ctx=ctx), reset_o)
nbytes = 2 * N * M * A * 8 + N * A * 8  # entries read + write, y rows
s = torch.randint(0, N, (16,), device="cuda")
e0, e1, ys = src[s].cpu().numpy(), ent[s].cpu().numpy(), y[s].cpu().numpy()
ok = bool(np.array_equal(e1, np.where(e0 > ys[:, None, :], e0, 0)))
print(json.dumps({"op": "orswot_forget_batch", "states": N, "members": M, "actors": A, "kernel_us": t * 1e6,
                  "GBs": nbytes / t / 1e9, "frac_of_8TBs": nbytes / t / 8e12,
                  "parity": "ok" if ok else "MISMATCH"}), flush=True)
del src, ent

# ---- Map<K, MVReg>
N, K, A, V = 16384, 1024, 32, 2
ec0 = torch.empty((N, K, A), dtype=torch.int64, device="cuda")
cg.synth_fill(ctx, ec0.view(N * K, A), 0x5EED0024, 0)
ec0.remainder_(64)
vc0 = torch.empty((N, K, V, A), dtype=torch.int64, device="cuda")
cg.synth_fill(ctx, vc0.view(N * K * V, A), 0x5EED0025, 0)
vc0.remainder_(64)
vv0 = torch.arange(N * K * V, device="cuda", dtype=torch.int64).view(N, K, V) + 1
ec, vc, vv = torch.empty_like(ec0), torch.empty_like(vc0), torch.empty_like(vv0)
mclock = torch.zeros((N, A), dtype=torch.int64, device="cuda")
ym = torch.empty((N, A), dtype=torch.int64, device="cuda")
cg.synth_fill(ctx, ym, 0x5EED0026, 0)
ym.remainder_(48)


def reset_m():
    ec.copy_(ec0)
    vc.copy_(vc0)
    vv.copy_(vv0)


t = timed("map_forget", lambda: cg.map.forget_batch(mclock, ec, vc, vv, ym, ctx=ctx), reset_m)
nbytes = 2 * (N * K * A * 8 + N * K * V * A * 8) + N * K * V * 8 + N * A * 8
s = torch.randint(0, N, (8,), device="cuda")
e0, e1, v0, v1 = ec0[s].cpu().numpy(), ec[s].cpu().numpy(), vc0[s].cpu().numpy(), vc[s].cpu().numpy()
yy = ym[s].cpu().numpy()
ef = np.where(e0 > yy[:, None, :], e0, 0)
alive = ef.any(axis=2)
vf = np.where(v0 > yy[:, None, None, :], v0, 0) * alive[:, :, None, None]
ok = bool(np.array_equal(e1, ef) and np.array_equal(v1, vf))
base = min(ec0.data_ptr(), ec.data_ptr())
print(json.dumps({"op": "map_forget_batch", "states": N, "keys": K, "actors": A, "vals": V, "kernel_us": t * 1e6,
                  "offsets_gib": {k: (v.data_ptr() - base) / 2**30 for k, v in (("ec0", ec0), ("vc0", vc0), ("ec", ec),
                                                                              ("vc", vc), ("vv", vv))},
                  "GBs": nbytes / t / 1e9, "frac_of_8TBs": nbytes / t / 8e12,
                  "parity": "ok" if ok else "MISMATCH"}), flush=True)
