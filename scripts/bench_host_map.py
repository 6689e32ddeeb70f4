"""Map<u32, MVReg<u64>> lub_many from HOST memory (CRDT_MEM_HOST) at BASELINE config-4 shape on one
MI355X: 16,384 replicas x 1,024 keys x 32 actors, V = 2 (12.25 GiB) in pinned host memory, streamed in
replica chunks through the two stage buffers (csrc/host_stage.hip: the running fold carried into the
next chunk as its replica 0, the exact left fold), against the pinned H2D rate of the same bytes and
the device-resident lub.  Parity: the host-mode result equals the device-resident lub of the same
replicas, every output word and every surviving deferred remove."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-crdt_amd"))

import crdts_gpu as cg  # noqa: E402
from crdts_gpu import host, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=16384)
ap.add_argument("--keys", type=int, default=1024)
ap.add_argument("--actors", type=int, default=32)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--stage-kb", type=int, default=262144)
args = ap.parse_args()
R, K, A, V = args.replicas, args.keys, args.actors, 2
T0 = time.time()


def log(msg):
    print(f"[{time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


torch.cuda.set_device(0)
ctx = cg.Context(0)
inp = synth.map_replicas(ctx, R, K, A, V, 0x5EED0004, kmax=256, p_def=0.1)
D = int(inp.def_off[-1])
names = ("clock", "ec", "vclk", "vval")
hs = {n: host.pinned_empty(tuple(getattr(inp, n).shape)) for n in names}
for n in names:
    torch.from_numpy(hs[n].view(np.int64)).copy_(getattr(inp, n))
drow = inp.def_row.cpu().numpy().astype(np.uint32)
dcl = inp.def_clock.cpu().numpy().view(np.uint64)
dks = inp.def_keys.cpu().numpy().view(np.uint64)
nbytes = sum(hs[n].nbytes for n in names)
log(f"generated {nbytes / 2**30:.2f} GiB in pinned host memory, {D} deferred removes")


def best(fn):
    ts = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), ts


def h2d():
    for n in names:
        getattr(inp, n).copy_(torch.from_numpy(hs[n].view(np.int64)), non_blocking=True)
    torch.cuda.synchronize()


t_h2d, _ = best(h2d)


def dev_lub():
    r = cg.map.lub_many(inp.clock, inp.ec, inp.vclk, inp.vval, def_off=inp.def_off, def_row=inp.def_row,
                        def_clock=inp.def_clock, def_keys=inp.def_keys, vout=4, ctx=ctx)
    torch.cuda.synchronize()
    return r


ref = dev_lub()
t_dev, _ = best(dev_lub)
hctx = host.HostContext(0, tune=f"stage_kb={args.stage_kb}")
got = None


def run_host():
    global got
    got = host.map_lub_many(hs["clock"], hs["ec"], hs["vclk"], hs["vval"], def_off=[0, D], def_row=drow,
                            def_clock=dcl, def_keys=dks, vout=4, ctx=hctx)


t_host, all_t = best(run_host)


def same(a, b):  # a host uint64 array, b the device int64 tensor of the same words
    return np.array_equal(np.asarray(a, dtype=np.uint64).reshape(-1), b.cpu().numpy().reshape(-1).view(np.uint64))


ok = (same(got.clock, ref.clock) and same(got.ec, ref.ec) and same(got.vclk, ref.vclk) and same(got.vval, ref.vval)
      and np.array_equal(got.nval.reshape(-1), ref.nval.cpu().numpy().reshape(-1).astype(np.uint32))
      and np.array_equal(got.def_keep, ref.def_keep.cpu().numpy().astype(np.uint8))
      and np.array_equal(got.def_keys, ref.def_keys.cpu().numpy().view(np.uint64)))
print(json.dumps({"op": "map_lub_many host (pinned, streamed)", "R": R, "K": K, "A": A, "V": V, "D": D, "bytes": nbytes,
                  "host_s": t_host, "host_runs_s": all_t, "host_GBs": nbytes / t_host / 1e9,
                  "h2d_pinned_s": t_h2d, "h2d_pinned_GBs": nbytes / t_h2d / 1e9, "frac_of_h2d": t_h2d / t_host,
                  "device_resident_s": t_dev, "replica_merges_per_s": R / t_host, "stage_kb": args.stage_kb,
                  "parity": "ok" if ok else "MISMATCH"}), flush=True)
sys.exit(0 if ok else 3)
