"""Host-memory mode (CRDT_MEM_HOST) throughput on one MI355X: the config-2 GCounter lub
(1M replicas x 256 actors, 2 GiB) and a pairwise merge_batch, starting from host arrays, against
the device-resident lub and the PCIe H2D rate of the same bytes.  Pageable and pinned
(crdt_host_alloc) inputs; chunk size sweep (tune key stage_kb).  Parity vs numpy each run."""
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
from crdts_gpu import host  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--replicas", type=int, default=1 << 20)
ap.add_argument("--actors", type=int, default=256)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--stage-kb", default="16384,65536,262144")
args = ap.parse_args()
R, A = args.replicas, args.actors
nbytes = R * A * 8

dev = torch.device("cuda", 0)
ctx = cg.Context(0)
rows_d = torch.empty((R, A), dtype=torch.int64, device=dev)
cg.synth_fill(ctx, rows_d, 0x5EED0002, 0)
pageable = rows_d.cpu().numpy().view(np.uint64)
pinned = host.pinned_empty((R, A))
pinned[...] = pageable
exp = pageable.max(axis=0)


def best(fn):
    fn()
    ts = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3


# device-resident lub and raw H2D for reference
out_d = torch.empty(A, dtype=torch.int64, device=dev)
ms_dev = best(lambda: (cg.gcounter.lub_many(rows_d, out=out_d, ctx=ctx), torch.cuda.synchronize()))
pin_t = torch.from_numpy(pinned.view(np.int64))
ms_h2d = best(lambda: (rows_d.copy_(pin_t, non_blocking=True), torch.cuda.synchronize()))
print(json.dumps({"op": "reference", "bytes": nbytes, "device_lub_ms": ms_dev, "h2d_pinned_ms": ms_h2d,
                  "h2d_pinned_GBs": nbytes / ms_h2d / 1e6}), flush=True)
ok = True
for kb in [int(x) for x in args.stage_kb.split(",")]:
    hctx = host.HostContext(0, tune=f"stage_kb={kb}")
    for name, arr in (("pageable", pageable), ("pinned", pinned)):
        got = host.lub_many("gcounter", arr, ctx=hctx)
        good = bool(np.array_equal(got, exp))
        ok = ok and good
        ms = best(lambda: host.lub_many("gcounter", arr, ctx=hctx))
        print(json.dumps({"op": "gcounter_lub_many_host", "input": name, "stage_kb": kb, "replicas": R, "actors": A,
                          "ms": ms, "GBs": nbytes / ms / 1e6, "replica_merges_per_s": R / ms * 1e3,
                          "vs_h2d_pinned": ms_h2d / ms, "parity": "ok" if good else "MISMATCH"}), flush=True)
    # pairwise merge of R/2 pairs from pinned host rows: 2 reads + 1 write of R/2 rows over PCIe
    half = R // 2
    s_rows = host.pinned_empty((half, A))
    s_rows[...] = pinned[:half]
    o_rows = pinned[half:2 * half]
    host.merge_batch("gcounter", s_rows, o_rows, ctx=hctx)
    good = bool(np.array_equal(s_rows, np.maximum(pinned[:half], o_rows)))
    ok = ok and good
    ms = best(lambda: host.merge_batch("gcounter", s_rows, o_rows, ctx=hctx))
    print(json.dumps({"op": "gcounter_merge_batch_host", "input": "pinned", "stage_kb": kb, "pairs": half, "actors": A,
                      "ms": ms, "GBs_moved": 3 * half * A * 8 / ms / 1e6, "pair_merges_per_s": half / ms * 1e3,
                      "parity": "ok" if good else "MISMATCH"}), flush=True)
    hctx.close()
    del s_rows
sys.exit(0 if ok else 3)
