"""Orswot lub_many from HOST memory (CRDT_MEM_HOST) at BASELINE config-3 shape on one MI355X:
65,536 replicas x 4,096 members x 64 actors (128 GiB of entries) in pinned host memory, streamed
in replica chunks through the two stage buffers (csrc/host_stage.hip orswot_lub_host_stream),
against the pinned H2D rate of the same bytes and the device-resident lub.  Parity: the host-mode
result equals the device-resident lub of the same replicas, every output word."""
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
ap.add_argument("--replicas", type=int, default=65536)
ap.add_argument("--members", type=int, default=4096)
ap.add_argument("--actors", type=int, default=64)
ap.add_argument("--gen-chunk", type=int, default=4096)
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--stage-kb", type=int, default=262144)
args = ap.parse_args()
R, M, A = args.replicas, args.members, args.actors
T0 = time.time()


def log(msg):
    print(f"[{time.time() - T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


torch.cuda.set_device(0)
ctx = cg.Context(0)
dev = torch.device("cuda", 0)
log(f"pinned host arrays: {R * (M + 1) * A * 8 / 2**30:.1f} GiB")
h_clock = host.pinned_empty((R, A))
h_entries = host.pinned_empty((R, M, A))
d_clock = torch.empty((R, A), dtype=torch.int64, device=dev)
d_entries = torch.empty((R, M, A), dtype=torch.int64, device=dev)
offs, dcls, dmems = [0], [], []
for r0 in range(0, R, args.gen_chunk):
    n = min(args.gen_chunk, R - r0)
    inp = synth.orswot_replicas(ctx, n, M, A, seed=0x5EED0003, kmax=48, first_row=r0, p_def=0.1,
                                clock=d_clock[r0:r0 + n], entries=d_entries[r0:r0 + n])
    torch.from_numpy(h_clock[r0:r0 + n].view(np.int64)).copy_(d_clock[r0:r0 + n])
    torch.from_numpy(h_entries[r0:r0 + n].view(np.int64)).copy_(d_entries[r0:r0 + n])
    dcls.append(inp.def_clock.cpu().numpy().view(np.uint64))
    dmems.append(inp.def_members.cpu().numpy().view(np.uint64))
    offs.append(offs[-1] + dcls[-1].shape[0])
log("generated")
dcl, dmem = np.concatenate(dcls), np.concatenate(dmems)
D = dcl.shape[0]
nbytes = R * (M + 1) * A * 8


def best(fn):
    ts = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), ts


# pinned H2D of the same bytes (into the device copy, in 8 GiB pieces)
def h2d():
    for r0 in range(0, R, args.gen_chunk):
        n = min(args.gen_chunk, R - r0)
        d_entries[r0:r0 + n].copy_(torch.from_numpy(h_entries[r0:r0 + n].view(np.int64)), non_blocking=True)
    d_clock.copy_(torch.from_numpy(h_clock.view(np.int64)), non_blocking=True)
    torch.cuda.synchronize()


t_h2d, _ = best(h2d)
log(f"h2d {t_h2d:.3f} s")
ref = cg.orswot.lub_many(d_clock, d_entries, def_off=[0, D], def_clock=torch.from_numpy(dcl.view(np.int64)).to(dev),
                         def_members=torch.from_numpy(dmem.view(np.int64)).to(dev), ctx=ctx)
torch.cuda.synchronize()
t_dev, _ = best(lambda: (cg.orswot.lub_many(d_clock, d_entries, def_off=[0, D],
                                            def_clock=torch.from_numpy(dcl.view(np.int64)).to(dev),
                                            def_members=torch.from_numpy(dmem.view(np.int64)).to(dev), ctx=ctx),
                         torch.cuda.synchronize()))
hctx = host.HostContext(0, tune=f"stage_kb={args.stage_kb}")
got = None


def run_host():
    global got
    got = host.orswot_lub_many(h_clock, h_entries, def_off=[0, D], def_clock=dcl, def_members=dmem, ctx=hctx)


t_host, all_t = best(run_host)
ok = (np.array_equal(got.clock, ref.clock.cpu().numpy().view(np.uint64))
      and np.array_equal(got.entries, ref.entries.cpu().numpy().view(np.uint64))
      and np.array_equal(got.def_keep, ref.def_keep.cpu().numpy().astype(np.uint8)))
print(json.dumps({"op": "orswot_lub_many host (pinned, streamed)", "R": R, "M": M, "A": A, "D": D, "bytes": nbytes,
                  "host_s": t_host, "host_runs_s": all_t, "host_GBs": nbytes / t_host / 1e9,
                  "h2d_pinned_s": t_h2d, "h2d_pinned_GBs": nbytes / t_h2d / 1e9, "frac_of_h2d": t_h2d / t_host,
                  "device_resident_s": t_dev, "replica_merges_per_s": R / t_host, "stage_kb": args.stage_kb,
                  "parity": "ok" if ok else "MISMATCH"}), flush=True)
sys.exit(0 if ok else 3)
