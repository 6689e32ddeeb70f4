"""Diagnose a Map GPU parity failure: one op-replay case under several tune settings."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-crdt_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import oracle as O, crdts_gpu as cg
from gpu_util import to_dev, to_host
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 1
rng = np.random.default_rng(seed)
K, A = int(rng.integers(1, 70)), int(rng.integers(1, 9))
R = int(rng.integers(1, 40))
p_rm = float(rng.choice([0.15, 0.3, 0.45]))
maps = O.gen_map_replicas(seed, R, K, A, steps=int(rng.integers(20, 300)), p_rm=p_rm, p_up=0.7 - p_rm)
V = O.max_vals(maps)
d = O.map_to_dense(maps, K, A, V)
vout = 8
exp = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], d["def_row"], d["def_clock"], d["def_keys"], vout)
print("K", K, "A", A, "R", R, "V", V, "D", len(d["def_row"]), "exp nval max", exp[4].max())
torch.cuda.set_device(0)
for spec in ["mspec=1", "mspec=0", "mglds=0,mspec=1", "mglds=0,mspec=0"]:
    ctx = cg.Context(0)
    ctx.tune(spec)
    res = cg.map.lub_many(to_dev(d["clock"]), to_dev(d["ec"]), to_dev(d["vclk"]), to_dev(d["vval"]), vout=vout, ctx=ctx, check=False)
    ge, gv, gvv, gn = to_host(res.ec), to_host(res.vclk), to_host(res.vval), res.nval.cpu().numpy()
    bad = [k for k in range(K) if not (np.array_equal(ge[k], exp[1][k]) and np.array_equal(gv[k], exp[2][k]) and np.array_equal(gvv[k], exp[3][k]) and gn[k] == exp[4][k])]
    print(spec, "flags", int(res.flags.max()), "bad keys", bad[:10])
    for k in bad[:2]:
        print("  key", k, "gpu n", gn[k], "exp n", exp[4][k])
        print("   gpu ec", ge[k].tolist(), "exp", exp[1][k].tolist())
        print("   gpu vals", [(gv[k, s].tolist(), int(gvv[k, s])) for s in range(gn[k])])
        print("   exp vals", [(exp[2][k, s].tolist(), int(exp[3][k, s])) for s in range(exp[4][k])])
