"""Map forget run-to-run / process-to-process spread: the bench_forget.py Map
workload (16,384 states x 1,024 keys x 32 actors x V=2), timed per launch over many reps in one
process, with the state buffers either as separate torch allocations (as before) or carved from
ONE slab allocation (--slab), and the base-address alignment of each buffer recorded.  Run it in
several processes to see whether the spread follows the allocation layout."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-crdt_amd")]
import crdts_gpu as cg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--slab", action="store_true")
ap.add_argument("--carve-gib", type=int, default=0,
                help="carve the state buffers from ONE allocation of this many GiB (>= 13), as "
                     "scripts/bench_forget.py's Map buffers end up inside the freed 32 GiB Orswot segment")
ap.add_argument("--reps", type=int, default=15)
ap.add_argument("--tag", default="")
ap.add_argument("--reset", choices=["synth", "copy"], default="synth",
                help="synth: regenerate the states before each launch; copy: copy them from pristine "
                     "tensors as scripts/bench_forget.py does")
ap.add_argument("--offset-gib", type=float, default=0.0, help="with --carve-gib: offset of the state buffers in it")
ap.add_argument("--orswot-first", action="store_true",
                help="run bench_forget.py's Orswot forget workload (32 GiB states) before the Map one")
args = ap.parse_args()
torch.cuda.set_device(0)
ctx = cg.Context(0)
if args.orswot_first:  # as scripts/bench_forget.py: Orswot 16,384 x 4,096 x 64 forget, 6 launches, then freed
    No, Mo, Ao = 16384, 4096, 64
    src = torch.empty((No, Mo, Ao), dtype=torch.int64, device="cuda")
    cg.synth_fill(ctx, src.view(No * Mo, Ao), 0x5EED0021, 0)
    src.remainder_(64)
    ent = torch.empty_like(src)
    oc = torch.empty((No, Ao), dtype=torch.int64, device="cuda")
    cg.synth_fill(ctx, oc, 0x5EED0022, 0)
    oy = torch.empty((No, Ao), dtype=torch.int64, device="cuda")
    cg.synth_fill(ctx, oy, 0x5EED0023, 0)
    for _ in range(6):
        ent.copy_(src)
        cg.orswot.forget_batch(oc, ent, oy, ctx=ctx)
    torch.cuda.synchronize()
    del src, ent
N, K, A, V = 16384, 1024, 32, 2
n_ec, n_vc, n_vv = N * K * A, N * K * V * A, N * K * V
if args.carve_gib:
    slab = torch.empty(args.carve_gib << 27, dtype=torch.int64, device="cuda")
    o = int(args.offset_gib * (1 << 27))
    ec = slab[o:o + n_ec].view(N, K, A)
    vc = slab[o + n_ec:o + n_ec + n_vc].view(N, K, V, A)
    vv = slab[o + n_ec + n_vc:o + n_ec + n_vc + n_vv].view(N, K, V)
elif args.slab:
    slab = torch.empty(n_ec + n_vc + n_vv, dtype=torch.int64, device="cuda")
    ec = slab[:n_ec].view(N, K, A)
    vc = slab[n_ec:n_ec + n_vc].view(N, K, V, A)
    vv = slab[n_ec + n_vc:].view(N, K, V)
else:
    ec = torch.empty((N, K, A), dtype=torch.int64, device="cuda")
    vc = torch.empty((N, K, V, A), dtype=torch.int64, device="cuda")
    vv = torch.empty((N, K, V), dtype=torch.int64, device="cuda")
# the synthetic content is regenerated before every rep (no second copy of 12 GiB held)
mclock = torch.zeros((N, A), dtype=torch.int64, device="cuda")
ym = torch.empty((N, A), dtype=torch.int64, device="cuda")
cg.synth_fill(ctx, ym, 0x5EED0026, 0)
ym.remainder_(48)


def regen():
    cg.synth_fill(ctx, ec.view(N * K, A), 0x5EED0024, 0)
    ec.remainder_(64)
    cg.synth_fill(ctx, vc.view(N * K * V, A), 0x5EED0025, 0)
    vc.remainder_(64)
    torch.arange(1, n_vv + 1, device="cuda", dtype=torch.int64, out=vv.view(-1))


if args.reset == "copy":
    regen()
    ec0, vc0, vv0 = ec.clone(), vc.clone(), vv.clone()

    def reset():
        ec.copy_(ec0)
        vc.copy_(vc0)
        vv.copy_(vv0)
else:
    reset = regen


times = []
for r in range(args.reps + 1):
    reset()
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    cg.map.forget_batch(mclock, ec, vc, vv, ym, ctx=ctx)
    torch.cuda.synchronize()
    ctx.set_timing(False)
    ms, n = ctx.timing("map_forget")
    if r:
        times.append(ms / n)
nbytes = 2 * (n_ec * 8 + n_vc * 8) + n_vv * 8 + N * A * 8
t = np.array(times)
align = {k: {"mod_2MiB": p % (2 << 20), "mod_1GiB": p % (1 << 30)} for k, p in
         (("ec", ec.data_ptr()), ("vc", vc.data_ptr()), ("vv", vv.data_ptr()))}
print(json.dumps({"op": "map_forget_spread", "tag": args.tag, "slab": args.slab, "carve_gib": args.carve_gib,
                  "orswot_first": args.orswot_first, "offset_gib": args.offset_gib,
                  "reset": args.reset, "reps": args.reps,
                  "ms_min": float(t.min()), "ms_median": float(np.median(t)), "ms_max": float(t.max()),
                  "GBs_median": nbytes / np.median(t) / 1e6, "ms_all": [round(x, 4) for x in t.tolist()],
                  "align": align}), flush=True)
