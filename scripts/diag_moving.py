"""Diagnostic: tests/test_gpu_qhull_c3.py::test_speculative_builds_moving_swarm
step by step — the swarm at x0, x0, x1, x0 through one context, each step's
records against the oracle at its own state; per step the fields that differ,
and for the differing pairs the GPU's n_reach / flags against both oracle
states.  usage: diag_moving.py [reps] (LQRO_* schedule variables as the test)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lqr-obstacles_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import lqro  # noqa: E402
import pyoracle as oracle  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
g = oracle.synthesize()
N, H = 1024, 100
x0, vg = lqro.synthetic_swarm(N)
x1 = x0.copy()
x1[:, 0:3] += 1.0 * x0[:, 3:6]
T, NCF = oracle.tables(g["A"], g["B"], g["L"], g["E"], H)
ref = []
oracle.set_hull_rule(1, round16=True)
for x in (x0, x1):
    oracle.carry_normal(np.zeros(3))
    rv, rr = oracle.step(T, NCF, oracle.sphere(100), x, vg, threads=16)
    ref.append((rv, rr))
oracle.set_hull_rule(0)
print("oracle done", flush=True)
F = ("n_reach", "reach_hash", "flags", "facet", "dist", "plane_point", "plane_normal")
for rep in range(reps):
    ctx = lqro.Context(lqro.config(N, H, 100, flags=lqro.LQRO_FLAG_RECORDS | lqro.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(g["A"], g["B"], g["L"], g["E"])
    for t, (x, s) in enumerate([(x0, 0), (x0, 0), (x1, 1), (x0, 0)]):
        ctx.carry_normal(np.zeros(3))
        try:
            v = ctx.step(x, vg)
        except lqro.QhullMergeSuspect as e:
            print(f"    (merge suspect: {e.pairs})")
            v = e.newv
        r = ctx.records()
        rr, ro = ref[s][1], ref[1 - s][1]
        bad = {}
        for f in F:
            a, b = r[f], rr[f]
            if f == "flags":
                a = a & ~lqro.REC_LOCAL
            d = ~np.all((a == b).reshape(len(a), -1), axis=1) if a.ndim > 1 else a != b
            if a.dtype.kind == "f":
                d = ~np.all((a.view(np.uint32 if a.dtype.itemsize == 4 else np.uint64) ==
                             b.view(np.uint32 if b.dtype.itemsize == 4 else np.uint64)).reshape(len(a), -1), axis=1)
            if d.any():
                bad[f] = np.nonzero(d)[0]
        vok = np.array_equal(v.view(np.uint64), ref[s][0].view(np.uint64))
        print(f"rep {rep} step {t}: " + (", ".join(f"{f} {len(ix)}" for f, ix in bad.items()) or "records equal") +
              f"; newV {'equal' if vok else 'DIFFERS'}; stats {ctx.stats()}", flush=True)
        ix = np.unique(np.concatenate(list(bad.values()))) if bad else []
        for k in ix[:12]:
            print(f"    pair {k} ({r['i'][k]}, {r['j'][k]}): gpu n_reach {r['n_reach'][k]} flags {r['flags'][k]:#x}; "
                  f"oracle here {rr['n_reach'][k]} {rr['flags'][k]:#x}; other state {ro['n_reach'][k]} "
                  f"{ro['flags'][k]:#x}")
    ctx.close()
