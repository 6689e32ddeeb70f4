"""Causal helpers at config-2 scale on one MI355X: glb / forget / partial_cmp of 1,048,576 row
pairs x 256 actors, GCounter / PNCounter read of 1,048,576 rows, and the all-pairs partial_cmp
matrix of 4,096 clocks x 64 actors.  HIP-event kernel time, algorithmic bytes (or compares),
parity of a row sample against the oracle.  One JSON line per op."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-crdt_amd"), os.path.join(ROOT, "oracle")]
import crdts_gpu as cg  # noqa: E402

N, A = 1 << 20, 256
torch.cuda.set_device(0)
ctx = cg.Context(0)
x = torch.empty((N, A), dtype=torch.int64, device="cuda")
y = torch.empty((N, A), dtype=torch.int64, device="cuda")
cg.synth_fill(ctx, x, 0x5EED0006, 0)
cg.synth_fill(ctx, y, 0x5EED0007, 0)
out = torch.empty_like(x)
torch.cuda.synchronize()


def timed(name, fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    ctx.timing_reset()
    ctx.set_timing(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    ms, n = ctx.timing(name)
    ctx.set_timing(False)
    t = ms / n / 1e3
    return {"kernel_us": t * 1e6, "GBs": nbytes / t / 1e9, "frac_of_8TBs": nbytes / t / 8e12}


import oracle as O  # noqa: E402  (checker only)

res = []
row = N * A * 8
r = timed("pair_op", lambda: cg.causal.glb(x, y, out=out, ctx=ctx), 3 * row)
s = np.random.default_rng(0).choice(N, 64, replace=False)
xs, ys, os_ = (t[torch.from_numpy(s).cuda()].cpu().numpy().view(np.uint64) for t in (x, y, out))
ok = all(np.array_equal(os_[i], np.minimum(xs[i], ys[i])) for i in range(64))
res.append(dict(op="glb", rows=N, actors=A, parity="ok" if ok else "MISMATCH", **r))
r = timed("pair_op", lambda: cg.causal.forget(x, y, out=out, ctx=ctx), 3 * row)
os_ = out[torch.from_numpy(s).cuda()].cpu().numpy().view(np.uint64)
ok = all(np.array_equal(os_[i], np.where(xs[i] > ys[i], xs[i], 0)) for i in range(64))
res.append(dict(op="forget", rows=N, actors=A, parity="ok" if ok else "MISMATCH", **r))
cmpres = {}
r = timed("pair_cmp", lambda: cmpres.__setitem__("v", cg.causal.partial_cmp(x, y, ctx=ctx)), 2 * row + N)
c = cmpres["v"][torch.from_numpy(s).cuda()].cpu().numpy()
codes = {O.EQUAL: 0, O.GREATER: 1, O.LESS: -1, O.NONE: 2}
vc = lambda r_: O.VClock({a: int(v) for a, v in enumerate(r_) if v})  # noqa: E731
ok = all(c[i] == codes[vc(xs[i]).partial_cmp(vc(ys[i]))] for i in range(64))
res.append(dict(op="partial_cmp", rows=N, actors=A, parity="ok" if ok else "MISMATCH", **r))
rd = {}
r = timed("read_sum", lambda: rd.__setitem__("v", cg.causal.read_sums("gcounter", x, ctx=ctx)), row + 16 * N)
w = rd["v"][torch.from_numpy(s).cuda()]
ok = cg.causal.words_to_ints(w, False) == [sum(int(v) for v in xs[i]) for i in range(64)]
res.append(dict(op="gcounter_read", rows=N, actors=A, parity="ok" if ok else "MISMATCH", **r))
Nm, Am = 4096, 64
m_in = x[:Nm, :Am].contiguous()
mres = {}
r = timed("cmp_matrix", lambda: mres.__setitem__("v", cg.causal.cmp_matrix(m_in, ctx=ctx)), Nm * Nm)
mm = mres["v"][:64, :64].cpu().numpy()
b = m_in[:64].cpu().numpy().view(np.uint64)
ok = all(mm[i, j] == codes[vc(b[i]).partial_cmp(vc(b[j]))] for i in range(64) for j in range(64))
res.append(dict(op="cmp_matrix", clocks=Nm, actors=Am, pairs=Nm * Nm, parity="ok" if ok else "MISMATCH",
                kernel_us=r["kernel_us"], pair_compares_per_s=Nm * Nm / (r["kernel_us"] / 1e6)))
# batched apply: 64M GCounter dots scattered over the 1M x 256 states (random cells)
n_ops = 1 << 26
g = torch.Generator(device="cuda")
g.manual_seed(7)
si = torch.randint(0, N, (n_ops,), device="cuda", dtype=torch.int32, generator=g)
ac = torch.randint(0, A, (n_ops,), device="cuda", dtype=torch.int32, generator=g)
ct = torch.randint(0, 1 << 40, (n_ops,), device="cuda", dtype=torch.int64, generator=g)
before = x[si[:64].long(), ac[:64].long()].clone()
r = timed("apply", lambda: cg.apply.apply_dots("gcounter", x, si, ac, ct, ctx=ctx), n_ops * 16)
after = x[si[:64].long(), ac[:64].long()]
ok = bool(((after.cpu().numpy().view(np.uint64) >= ct[:64].cpu().numpy().view(np.uint64)).all()))
res.append(dict(op="gcounter_apply", states=N, actors=A, ops=n_ops, parity="ok" if ok else "MISMATCH",
                kernel_us=r["kernel_us"], ops_per_s=n_ops / (r["kernel_us"] / 1e6)))
for d in res:
    d["tune"] = os.environ.get("CRDT_TUNE", "")
    print(json.dumps(d), flush=True)
sys.exit(0 if all(d["parity"] == "ok" for d in res) else 3)
