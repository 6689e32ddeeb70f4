"""Replays the reference's known-answer tests (tests/golden/kat_*.json).

`merge_hook(dst_obj, src_obj, kind) -> new_dst_obj` lets the GPU tests route every merge
through libcrdt_gpu; by default the oracle's own merge runs.  `causal_hook` (optional) routes
VClock forget / glb / partial_cmp and counter read() the same way: an object with methods
forget(x, y) / glb(x, y) (mutate x), cmp(x, y) -> Ordering code or None, read(counter) -> int.
`apply_hook(state, op)` applies an Orswot op built by the reference's ctx API (add / rm steps)
to `state` in place (default: the oracle's own CmRDT::apply).
"""
import json
import os

import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_cases(fname):
    with open(os.path.join(GOLDEN, fname)) as f:
        return json.load(f)["cases"]


def _vc(pairs):
    return O.VClock({a: c for a, c in pairs})


def _new(kind):
    return {"vclock": O.VClock, "gcounter": O.GCounter, "pncounter": O.PNCounter,
            "gset": O.GSet, "orswot": O.Orswot, "mvreg": O.MVReg}[kind]()


def _clone(x):
    if isinstance(x, O.VClock):
        return x.copy()
    if isinstance(x, O.Orswot):
        return x.copy()
    if isinstance(x, O.GCounter):
        c = O.GCounter(); c.inner = x.inner.copy(); return c
    if isinstance(x, O.PNCounter):
        c = O.PNCounter(); c.p.inner = x.p.inner.copy(); c.n.inner = x.n.inner.copy(); return c
    if isinstance(x, O.GSet):
        return O.GSet(x.value)
    if isinstance(x, O.LWWReg):
        return O.LWWReg(x.val, x.marker)
    if isinstance(x, O.MVReg):
        return x.copy()
    if isinstance(x, (O.ReadCtx, O.MVRegPut)):
        return x
    raise TypeError(type(x))


def kind_of(x):
    for k, t in (("vclock", O.VClock), ("gcounter", O.GCounter), ("pncounter", O.PNCounter),
                 ("gset", O.GSet), ("orswot", O.Orswot), ("lwwreg", O.LWWReg), ("mvreg", O.MVReg)):
        if isinstance(x, t):
            return k
    raise TypeError(type(x))


def default_merge(dst, src, kind):
    if kind == "lwwreg":
        dst.merge(_clone(src))
    else:
        dst.merge(_clone(src))
    return dst


def _cmp(x, op, y):
    if op == "==":
        return x == y
    if op == "!=":
        return x != y
    if op == ">":
        return x > y
    if op == "<":
        return x < y
    if op == "!>":
        return not (x > y)
    if op == "!<":
        return not (x < y)
    if op == "||":
        return x.concurrent(y)
    raise ValueError(op)


def default_apply(v, op):
    v.apply(op)


def run_case(case, merge_hook=default_merge, causal_hook=None, apply_hook=default_apply):
    env = {}
    for st in case["steps"]:
        op, args = st[0], st[1:]
        if op == "new":
            env[args[0]] = _new(args[1])
        elif op == "new_lww":
            env[args[0]] = O.LWWReg(args[1], args[2])
        elif op == "clone":
            env[args[0]] = _clone(env[args[1]])
        elif op == "vc_apply":
            env[args[0]].apply(O.Dot(args[1], args[2]))
        elif op == "vc_inc":
            v = env[args[0]]
            v.apply(v.inc(args[1]))
        elif op == "inc":
            v = env[args[0]]
            v.apply(v.inc(args[1]))
        elif op == "dec":
            v = env[args[0]]
            v.apply(v.dec(args[1]))
        elif op == "insert":
            env[args[0]].insert(args[1])
        elif op == "merge":
            dst, src = env[args[0]], env[args[1]]
            env[args[0]] = merge_hook(dst, src, kind_of(dst))
        elif op == "forget":
            if causal_hook is not None and isinstance(env[args[0]], O.VClock):
                causal_hook.forget(env[args[0]], env[args[1]])
            else:
                env[args[0]].forget(env[args[1]])
        elif op == "glb":
            if causal_hook is not None:
                causal_hook.glb(env[args[0]], env[args[1]])
            else:
                env[args[0]].glb(env[args[1]])
        elif op == "update":
            reg, val, marker, expect_err = env[args[0]], args[1], args[2], args[3]
            try:
                reg.update(val, marker)
                err = False
            except O.ConflictingMarker:
                err = True
            assert err == expect_err, f"update({val},{marker}) err={err}"
        elif op == "merge_err":
            dst, src, expect_err = env[args[0]], env[args[1]], args[2]
            try:
                env[args[0]] = merge_hook(dst, src, "lwwreg")
                err = False
            except O.ConflictingMarker:
                err = True
            assert err == expect_err
        elif op == "add":
            v = env[args[0]]
            apply_hook(v, v.add(args[1], v.read().derive_add_ctx(args[2])))
        elif op == "rm":
            v = env[args[0]]
            apply_hook(v, v.rm(args[1], v.contains(args[1]).derive_rm_ctx()))
        elif op == "rm_clock":
            v = env[args[0]]
            apply_hook(v, v.rm(args[1], O.RmCtx(_vc(args[2]))))
        elif op == "save_read":
            env[args[0]] = env[args[1]].read()
        elif op == "save_contains":
            env[args[0]] = env[args[1]].contains(args[2])
        elif op == "add_ctx":
            v, ctx = env[args[0]], env[args[2]]
            apply_hook(v, v.add(args[1], ctx.derive_add_ctx(args[3])))
        elif op == "rm_ctx":
            v, ctx = env[args[0]], env[args[2]]
            apply_hook(v, v.rm(args[1], ctx.derive_rm_ctx()))
        elif op == "assert_add_op":
            v = env[args[0]]
            opv = v.add(args[1], v.read().derive_add_ctx(args[2]))
            assert opv.dot == O.Dot(args[3][0], args[3][1]) and opv.members == {args[1]}
        elif op == "assert_dots":
            assert env[args[0]] == _vc(args[1]), (env[args[0]], args[1])
        elif op == "assert_get":
            assert env[args[0]].get(args[1]) == args[2]
        elif op == "assert_cmp":
            assert _cmp(env[args[0]], args[1], env[args[2]]), st
            if causal_hook is not None and isinstance(env[args[0]], O.VClock):
                assert causal_hook.cmp(env[args[0]], env[args[2]]) == env[args[0]].partial_cmp(env[args[2]]), st
        elif op == "assert_read":
            v = env[args[0]]
            if isinstance(v, (O.GCounter, O.PNCounter)):
                assert v.read() == args[1], (v.read(), args[1])
                if causal_hook is not None:
                    assert causal_hook.read(v) == args[1], (causal_hook.read(v), args[1])
            elif isinstance(v, O.GSet):
                assert v.value == set(args[1])
            else:
                assert v.read().val == set(args[1]), (v.read().val, args[1])
        elif op == "assert_read_eq":
            assert env[args[0]].read() == env[args[1]].read()
        elif op == "assert_read_gt":
            assert env[args[0]].read() > env[args[1]].read()
        elif op == "assert_contains":
            v = env[args[0]]
            got = v.contains(args[1])
            got = got.val if isinstance(got, O.ReadCtx) else got
            assert got == args[2]
        elif op == "assert_contains_rm_clock":
            assert env[args[0]].contains(args[1]).rm_clock == _vc(args[2])
        elif op == "assert_rm_clock":
            assert env[args[0]].rm_clock == _vc(args[1])
        elif op == "assert_add_clock":
            assert env[args[0]].add_clock == _vc(args[1])
        elif op == "assert_read_add_clock":
            assert env[args[0]].read().add_clock == _vc(args[1])
        elif op == "assert_deferred_len":
            assert len(env[args[0]].deferred) == args[1], env[args[0]].deferred
        elif op == "mv_write":  # reg.apply(reg.write(val, reg.read().derive_add_ctx(actor)))
            v = env[args[0]]
            apply_hook(v, v.write(args[1], v.read().derive_add_ctx(args[2])))
        elif op == "mv_write_from":  # dst.apply(src.write(val, src.read().derive_add_ctx(actor)))
            dst, src = env[args[0]], env[args[1]]
            apply_hook(dst, src.write(args[2], src.read().derive_add_ctx(args[3])))
        elif op == "mv_put":  # reg.apply(Op::Put { clock, val })
            apply_hook(env[args[0]], O.MVRegPut(_vc(args[1]), args[2]))
        elif op == "save_mv_write_ctx":  # op = reg.write(val, ctx.derive_add_ctx(actor))
            env[args[0]] = env[args[1]].write(args[2], env[args[3]].derive_add_ctx(args[4]))
        elif op == "apply_op":
            apply_hook(env[args[0]], env[args[1]])
        elif op == "assert_mv_vals":
            assert env[args[0]].read().val == args[1], (env[args[0]].read().val, args[1])
        elif op == "assert_mv_vals_any":
            assert env[args[0]].read().val in args[1], (env[args[0]].read().val, args[1])
        elif op == "assert_eq":
            assert env[args[0]] == env[args[1]], (env[args[0]], env[args[1]])
        elif op == "assert_eq_new":
            assert env[args[0]] == _new(args[1]), env[args[0]]
        elif op == "assert_lww":
            assert env[args[0]] == O.LWWReg(args[1], args[2]), env[args[0]]
        else:
            raise ValueError(f"unknown step {op}")
    return env
