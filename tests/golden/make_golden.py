"""Writes tests/golden/synth.json: small fixtures of the counter-based synthetic generators
(crdt_synth_fill kinds 0-3, crdt_synth_orswot, crdt_synth_map) as restated by the oracle
(oracle/oracle.py synth_*), plus the oracle's folds of two of them.  The CPU suite checks the
restatement against this file (tests/test_golden_synth.py) and the GPU suite checks the device
generators against it, so any drift of either side is caught.  Re-run only when a generator is
changed on purpose:  python tests/golden/make_golden.py"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402

# every case: (name, parameters); values are stored as decimal strings (u64 does not fit JSON ints)
FILL = [dict(seed=0x5EED0002, rows=4, width=8, first_row=3, kind=k) for k in range(4)]
ORSWOT = dict(seed=0x5EED0003, R=4, M=16, A=5, kmax=12, row0=2)
MAP = dict(seed=0x5EED0004, R=5, K=10, A=4, V=2, kmax=9, p_def=0.5)


def s(a):
    return [str(int(x)) for x in np.asarray(a, np.uint64).ravel()]


def build():
    out = {"fill": [], "orswot": None, "map": None}
    for p in FILL:
        m = O.synth_matrix(p["seed"], p["rows"], p["width"], p["kind"], row0=p["first_row"])
        out["fill"].append(dict(p, values=s(m)))
    c, e = O.synth_orswot(ORSWOT["seed"], ORSWOT["R"], ORSWOT["M"], ORSWOT["A"], ORSWOT["kmax"], row0=ORSWOT["row0"])
    fc, fe = O.dense_orswot_join_fold(c, e)
    out["orswot"] = dict(ORSWOT, clock=s(c), entries=s(e), fold_clock=s(fc), fold_entries=s(fe))
    p = MAP
    dfr = O.synth_map_deferred(p["seed"], p["R"], p["K"], p["A"], p["kmax"], p_def=p["p_def"])
    d = O.synth_map(p["seed"], p["R"], p["K"], p["A"], p["V"], p["kmax"], deferred=dfr)
    f = O.map_fold(d["clock"], d["ec"], d["vclk"], d["vval"], dfr[0], dfr[1], dfr[2], 4)
    out["map"] = dict(p, **{k: s(d[k]) for k in ("clock", "ec", "vclk", "vval")},
                      def_row=s(dfr[0]), def_clock=s(dfr[1]), def_keys=s(dfr[2]),
                      fold_clock=s(f[0]), fold_ec=s(f[1]), fold_vclk=s(f[2]), fold_vval=s(f[3]), fold_nval=s(f[4]))
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "synth.json"), "w") as fh:
        json.dump(build(), fh, indent=0)
    print("wrote", os.path.join(HERE, "synth.json"))
