"""Experiment (round 5): does the placement of BASELINE config 3's 128 GiB input change the Orswot
join's time?  The same synthetic replicas are generated into (a) a torch caching-allocator block and
(b) one hipExtMallocWithFlags(hipDeviceMallocContiguous) block, and the fold is timed on each with
the context's HIP-event timer.  Output: one JSON line per placement.  Not part of the product."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-crdt_amd")]
import crdts_gpu as cg  # noqa: E402
from crdts_gpu import _abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--order", default="contig,torch")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--replicas", type=int, default=65536)
args = ap.parse_args()
R, M, A, kmax, p_def, seed = args.replicas, 4096, 64, 48, 0.1, 0x5EED0003

torch.cuda.set_device(0)
ctx = cg.Context(0)
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
CONTIG = 0x4


def run(mode):
    nc, ne = R * A * 8, R * M * A * 8
    keep = []
    if mode == "torch":
        c = torch.empty((R, A), dtype=torch.int64, device="cuda")
        e = torch.empty((R, M, A), dtype=torch.int64, device="cuda")
        keep = [c, e]
        pc, pe = c.data_ptr(), e.data_ptr()
    else:
        bc, be = ctypes.c_void_p(), ctypes.c_void_p()
        rc1 = hip.hipExtMallocWithFlags(ctypes.byref(bc), nc, CONTIG)
        rc2 = hip.hipExtMallocWithFlags(ctypes.byref(be), ne, CONTIG)
        if rc1 or rc2:
            print(json.dumps({"mode": mode, "error": [rc1, rc2]}), flush=True)
            for b in (bc, be):
                if b.value:
                    hip.hipFree(b)
            return
        pc, pe = bc.value, be.value
    torch.cuda.synchronize()
    ctx.call("crdt_synth_orswot", ctypes.c_void_p(pc), ctypes.c_void_p(pe), R, M, A, 0,
             ctypes.c_uint64(seed), ctypes.c_uint64(kmax))
    off, rows, rm, members = synth.orswot_deferred(seed, R, M, A, kmax, 0, p_def)
    D = rm.shape[0]
    dcl = torch.from_numpy(rm.view(np.int64)).cuda()
    dmem = torch.from_numpy(members.view(np.int64)).cuda()
    drow = torch.from_numpy(rows.astype(np.int32)).cuda()
    ctx.call("crdt_synth_orswot_rm", ctypes.c_void_p(pe), M, A, D, synth.dptr(drow), synth.dptr(dcl),
             synth.dptr(dmem))
    torch.cuda.synchronize()
    Mw = (M + 63) // 64
    oc = torch.empty((1, A), dtype=torch.int64, device="cuda")
    oe = torch.empty((1, M, A), dtype=torch.int64, device="cuda")
    kp = torch.empty(D, dtype=torch.uint8, device="cuda")
    mo = torch.empty((D, Mw), dtype=torch.int64, device="cuda")
    b = _abi.OrswotBatch()
    b.G, b.R, b.M, b.A = 1, R, M, A
    b.clock, b.clock_rstride, b.clock_gstride = pc, A, R * A
    b.entries = pe
    b.entry_mstride, b.entry_rstride, b.entry_gstride = A, M * A, R * M * A
    off_arr = (ctypes.c_size_t * 2)(0, D)
    b.def_off = ctypes.cast(off_arr, ctypes.POINTER(ctypes.c_size_t))
    b.def_clock, b.def_members = dcl.data_ptr(), dmem.data_ptr()
    o = _abi.OrswotOut()
    o.clock, o.entries = oc.data_ptr(), oe.data_ptr()
    o.def_keep, o.def_members = kp.data_ptr(), mo.data_ptr()
    ctx.call("crdt_orswot_lub_many", ctypes.byref(b), ctypes.byref(o))
    torch.cuda.synchronize()
    ref = (oc.sum().item(), oe.sum().item())
    ctx.timing_reset()
    ctx.set_timing(True)
    per = []
    for _ in range(args.reps):
        ctx.call("crdt_orswot_lub_many", ctypes.byref(b), ctypes.byref(o))
        torch.cuda.synchronize()
        ms, n = ctx.timing("orswot_join")
        per.append(ms / max(n, 1))
        ctx.timing_reset()
    ctx.set_timing(False)
    same = ref == (oc.sum().item(), oe.sum().item())
    alg = (R + 1) * (M * A + A) * 8
    best = min(per)
    print(json.dumps({"mode": mode, "pe": hex(pe), "kernel_ms": per, "frac_best": alg / (best / 1e3) / 8e12,
                      "repeatable": same}), flush=True)
    if mode != "torch":
        hip.hipFree(ctypes.c_void_p(pc))
        hip.hipFree(ctypes.c_void_p(pe))
    del keep
    torch.cuda.empty_cache()


for m in args.order.split(","):
    run(m)
