"""Measure the non-headline BASELINE configs and the other kernels on one MI355X.

  c1       VClock fold of 1,024 replicas x 64 actors (cache-resident, launch-bound) + the
           restated reference fold on one CPU core
  c5shard  one GPU's shard of config 5: 1,048,576 VClock replicas x 1,024 actors (8 GiB)
  gset     GSet lub, 1,048,576 replicas x 128 words (8,192-element universe)
  lww      LWWReg lub of 16,777,216 replicas (state + exact first conflict)
  merge    VClock merge_batch, 1,048,576 pairs x 256 actors (3 streams)
Each line: JSON with kernel time, GB/s of algorithmic bytes, replica-merges/s, parity."""
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
import oracle as O  # noqa: E402  (checker / CPU baseline only)

torch.cuda.set_device(0)
ctx = cg.Context(0)
SIGN = torch.tensor(-(2**63), dtype=torch.int64, device="cuda")
which = sys.argv[1:] or ["c1", "c5shard", "gset", "lww", "merge"]


def umax(t, dim):
    return (t ^ SIGN).amax(dim) ^ SIGN


def timed(fn, name, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ms, n = ctx.timing(name)
    ctx.set_timing(False)
    return wall, (ms / n / 1e3) if n else float("nan")


def emit(d):
    print(json.dumps(d), flush=True)


if "c1" in which:
    R, A = 1024, 64
    rows = O.synth_matrix(0x5EED0001, R, A, 0)
    x = torch.from_numpy(rows.view(np.int64)).cuda()
    out = torch.empty(A, dtype=torch.int64, device="cuda")
    wall, k = timed(lambda: cg.vclock.lub_many(x, out=out, ctx=ctx), "lub_stream", reps=200)
    exp, cpu_s = O.vclock_fold(rows)
    ok = np.array_equal(out.cpu().numpy().view(np.uint64), exp)
    cpu_reps = [O.vclock_fold(rows)[1] for _ in range(20)]
    emit({"config": "c1 vclock 1024x64", "wall_us": wall * 1e6, "kernel_us": k * 1e6,
          "replica_merges_per_s_gpu_wall": R / wall, "cpu_fold_s_median": float(np.median(cpu_reps)),
          "replica_merges_per_s_cpu_1core": R / float(np.median(cpu_reps)), "parity": ok,
          "note": "512 KiB input: launch-bound, not roofline-graded"})

if "c5shard" in which:
    R, A = 1 << 20, 1024
    x = torch.empty((R, A), dtype=torch.int64, device="cuda")
    cg.synth_fill(ctx, x, 0x5EED0005, 0)
    out = torch.empty(A, dtype=torch.int64, device="cuda")
    wall, k = timed(lambda: cg.vclock.lub_many(x, out=out, ctx=ctx), "lub_stream")
    ok = bool(torch.equal(out, umax(x, 0)))
    emit({"config": "c5 shard vclock 1048576x1024 (one GPU of 8)", "wall_us": wall * 1e6, "kernel_us": k * 1e6,
          "GBs": R * A * 8 / k / 1e9, "frac_of_8TBs": R * A * 8 / k / 8e12,
          "replica_merges_per_s": R / wall, "parity_vs_torch_umax": ok})
    del x

if "gset" in which:
    R, W = 1 << 20, 128
    x = torch.empty((R, W), dtype=torch.int64, device="cuda")
    cg.synth_fill(ctx, x, 0x5EED0006, 1)
    out = torch.empty(W, dtype=torch.int64, device="cuda")
    wall, k = timed(lambda: cg.gset.lub_many(x, out=out, ctx=ctx), "lub_stream")
    sample = O.synth_matrix(0x5EED0006, 4096, W, 1)
    h = out.cpu().numpy().view(np.uint64)
    ok = bool(((sample | h) == h).all())
    emit({"config": "gset 1048576x128 words", "kernel_us": k * 1e6, "GBs": R * W * 8 / k / 1e9,
          "frac_of_8TBs": R * W * 8 / k / 8e12, "replica_merges_per_s": R / wall,
          "parity_sampled_subset": ok})
    del x

if "lww" in which:
    R = 1 << 24
    m = torch.empty((1, R), dtype=torch.int64, device="cuda")
    v = torch.empty((1, R), dtype=torch.int64, device="cuda")
    cg.synth_fill(ctx, m, 0x5EED0007, 2)
    cg.synth_fill(ctx, v, 0x5EED0007, 3)
    res = [None]

    def run():
        res[0] = cg.lwwreg.lub_many(m, v, ctx=ctx)
    wall, k = timed(run, "lww_reduce")
    mh, vh = m.cpu().numpy().view(np.uint64)[0], v.cpu().numpy().view(np.uint64)[0]
    om, ov, of, cpu_s = O.lwwreg_fold(mh, vh)
    r = res[0]
    ok = (int(r.marker.cpu().numpy().view(np.uint64)[0]), int(r.val.cpu().numpy().view(np.uint64)[0]),
          int(r.first_conflict.cpu().numpy().view(np.uint64)[0])) == (om, ov, of)
    emit({"config": "lwwreg 16777216 replicas", "wall_us": wall * 1e6, "reduce_kernel_us": k * 1e6,
          "GBs_wall_2passes": 3 * R * 8 / wall / 1e9, "replica_merges_per_s": R / wall,
          "cpu_fold_replica_merges_per_s_1core": R / cpu_s, "parity": ok, "first_conflict": of})

if "merge" in which:
    N, A = 1 << 20, 256
    s = torch.empty((N, A), dtype=torch.int64, device="cuda")
    o = torch.empty((N, A), dtype=torch.int64, device="cuda")
    cg.synth_fill(ctx, s, 0x5EED0008, 0)
    cg.synth_fill(ctx, o, 0x5EED0009, 0)
    exp = torch.maximum(s ^ SIGN, o ^ SIGN) ^ SIGN
    cg.vclock.merge_batch(s, o, ctx=ctx)
    ok = bool(torch.equal(s, exp))
    wall, k = timed(lambda: cg.vclock.merge_batch(s, o, ctx=ctx), "merge_pairs")
    emit({"config": "vclock merge_batch 1048576 pairs x 256", "kernel_us": k * 1e6,
          "GBs": 3 * N * A * 8 / k / 1e9, "frac_of_8TBs": 3 * N * A * 8 / k / 8e12,
          "pair_merges_per_s": N / wall, "parity_vs_torch": ok})
