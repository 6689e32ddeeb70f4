"""Diagnose the ST (two waves per key) Map fold against the RS path and the oracle on the
old-heavy A = 32, V = 2 inputs of tests/test_gpu_map.py: per case, which keys differ and whether
repeated SP runs agree with each other (determinism)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("rust-crdt_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import crdts_gpu as cg  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_map import _gpu, _old_heavy  # noqa: E402
from gpu_util import to_host  # noqa: E402

torch.cuda.set_device(0)
ctxs = {}
for spec in ("mst=0", "mst=1"):
    c = cg.Context(0)
    c.tune(spec)
    ctxs[spec] = c


def run(ctx, d):
    res, _ = _gpu(ctx, d, 4)
    torch.cuda.synchronize()
    return {n: (to_host(getattr(res, n)) if n != "nval" else res.nval.cpu().numpy()) for n in ("clock", "ec", "vclk", "vval", "nval")}


bad = 0
cases = [(R, s) for R in (81, 17, 33, 65, 97, 145, 161) for s in range(6)]
for R, s in cases:
    rng = np.random.default_rng(4000 + R if s == 0 else 9000 + 100 * R + s)
    d = _old_heavy(rng, R, 8, 32)[0]
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"], 64)
    if int(exp[4].max() if exp[4].size else 0) > 4:
        continue
    exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"], 4)
    rs = run(ctxs["mst=0"], d)
    sps = [run(ctxs["mst=1"], d) for _ in range(3)]
    ok_rs = np.array_equal(rs["ec"], exp[1]) and np.array_equal(rs["vclk"], exp[2])
    det = all(all(np.array_equal(sps[0][n], x[n]) for n in x) for x in sps[1:])
    diff_keys = sorted({int(k) for x in sps for k in np.flatnonzero((x["ec"] != exp[1]).any(axis=1) | (x["vclk"] != exp[2]).reshape(8, -1).any(axis=1))})
    print(f"R={R} seed={s} D={d['def_row'].shape[0]} rs_ok={ok_rs} sp_deterministic={det} sp_bad_keys={diff_keys}", flush=True)
    if diff_keys:
        bad += 1
        k = diff_keys[0]
        x = sps[0]
        print("  key", k, "ec exp", exp[1][k].tolist(), flush=True)
        print("  key", k, "ec got", x["ec"][k].tolist(), flush=True)
        print("  rows with removes:", d["def_row"].tolist(), flush=True)
print("bad cases:", bad, "of", len(cases))
