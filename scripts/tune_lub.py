"""A/B the lattice lub launch geometry on the GPU (CRDT_TUNE knobs), one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-crdt_amd"))
import crdts_gpu as cg  # noqa: E402

R = 1 << 20
torch.cuda.set_device(0)
variants = [v for v in sys.argv[1:]] or [
    "interleave=0", "interleave=1", "interleave=1,bpc=4", "interleave=1,bpc=16", "interleave=1,unroll=4",
    "interleave=1,unroll=16", "interleave=1,bpc=4,unroll=16", "interleave=1,nt=0", "interleave=0,bpc=4",
    "interleave=1,bpc=2,unroll=16", "interleave=1,minsteps=64", "interleave=1,bpc=12"]
base = cg.Context(0)
g = torch.empty((R, 256), dtype=torch.int64, device="cuda")
p = torch.empty((R, 512), dtype=torch.int64, device="cuda")
cg.synth_fill(base, g, 0x5EED0002, 0)
cg.synth_fill(base, p, 0x5EED0003, 0)
ref_g = cg.gcounter.lub_many(g, ctx=base).clone()
ref_p = cg.pncounter.lub_many(p, ctx=base).clone()
og = torch.empty(256, dtype=torch.int64, device="cuda")
op = torch.empty(512, dtype=torch.int64, device="cuda")
res = []
for rep in range(2):
    for v in variants:
        os.environ["CRDT_TUNE"] = v
        ctx = cg.Context(0)
        out = {"tune": v, "rep": rep}
        for name, x, o, fn, ref in (("g", g, og, cg.gcounter.lub_many, ref_g), ("p", p, op, cg.pncounter.lub_many, ref_p)):
            for _ in range(3):
                fn(x, out=o, ctx=ctx)
            ctx.timing_reset()
            ctx.set_timing(True)
            for _ in range(20):
                fn(x, out=o, ctx=ctx)
            ms, n = ctx.timing("lub_stream")
            ctx.set_timing(False)
            assert torch.equal(o, ref), v
            out[name + "_us"] = round(ms / n * 1e3, 1)
            out[name + "_GBs"] = round(x.numel() * 8 / (ms / n * 1e-3) / 1e9, 1)
        ctx.close()
        res.append(out)
        print(json.dumps(out), flush=True)
