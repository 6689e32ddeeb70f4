"""Minimal driver for rocprofv3 passes over the Map fold kernel (config 4 shape by default)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-crdt_amd"))
import crdts_gpu as cg  # noqa: E402
from crdts_gpu import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=16384)
ap.add_argument("--keys", type=int, default=1024)
ap.add_argument("--actors", type=int, default=32)
ap.add_argument("--p-def", type=float, default=0.1)
ap.add_argument("--iters", type=int, default=3)
a = ap.parse_args()
torch.cuda.set_device(0)
ctx = cg.Context(0)
inp = synth.map_replicas(ctx, a.replicas, a.keys, a.actors, 2, 0x5EED0004, kmax=256, p_def=a.p_def)
for _ in range(a.iters):
    res = cg.map.lub_many(inp.clock, inp.ec, inp.vclk, inp.vval, def_off=inp.def_off, def_row=inp.def_row,
                          def_clock=inp.def_clock, def_keys=inp.def_keys, vout=4, ctx=ctx, check=False)
torch.cuda.synchronize()
print("done", int(res.flags.max().item()))
