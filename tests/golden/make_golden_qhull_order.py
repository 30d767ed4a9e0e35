#!/usr/bin/env python3
"""The reference's inside-hull rule with Qhull itself, over the reference's
whole pair loop.  TEST INFRASTRUCTURE, build container.

convexHull (LQRObstacles.cpp:867-969) writes the reachable points at 6
significant digits (:869-874), runs `qconvex n` and `qconvex Fv` (:879-880),
reads the planes as printed (%.16g, :895-899) and each facet's FIRST Fv
vertex at full precision (:925-939), and takes min_f |n_f . (vrel - P_f)|
over the facets in Qhull's order with a strict '<', writing `normal` only
when a facet after facet 0 wins (:955-968).  `normalVector` is declared
outside the t / i / j loops (:1385): a facet-0 win keeps the value the last
pair with more than 4 reachable points left (run_gjk's normal, or an earlier
hull's), across rows.

Here Qhull is scipy's qhull_r 2019.1 called exactly like qconvex
(tests/golden/qhull_lib.py; SURVEY §8c's stand-in for qconvex.exe), on the
points the oracle's pair body produces (pinned bit-exact to the reference's
own functions elsewhere: tests/test_oracle_vs_ref.py).  The loop below is the
reference's (t = one step, all rows, carried normal starting at 0); each
row's newV is the oracle's LP (pinned to the reference: newv.npz).

Stores tests/golden/qhull_order.npz:
  <w>_pairs: per inside-hull pair i, j, n_reach, facet count, the winning
      facet's index in Qhull's order and Fv triple, dist, normal (after the
      carry), stale flag;
  <w>_newv: every row's newV under the reference's rule;
  <w>_merged: per inside-hull pair whose qconvex output has a merged
      (non-simplicial) facet — Qhull's default pre-merge (C-0) — i, j, the
      merged hull's facet count, its non-simplicial facets' count and whether
      the winning facet is one of them; <w>_merged_facets: those facets'
      Fv lists (flattened, <w>_merged_offs: offsets per facet, per pair in
      <w>_merged_pairoffs), first vertex and plane (<w>_merged_planes);
  inject_*: six dense-swarm pairs with Qhull's full output (rounded points,
      Fv lists, planes as read back) for the GPU selection test hook.
and prints a summary (also to argv[1]).

Usage:  python tests/golden/make_golden_qhull_order.py [summary.json]
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "lqr-obstacles_amd")]
import pyoracle  # noqa: E402
import lqro  # noqa: E402  (the pure-Python swarm generator only)
import qhull_lib  # noqa: E402

WORKLOADS = (  # name, N, H, box, seed
    ("dense", 32, 45, 3.0, 11),
    ("c2", 64, 50, None, None),
    ("c3", 1024, 100, None, None),
    ("crowd22", 1024, 100, 22.0, 7),
)


def reference_hull(pts_full, vrel):
    """LQRO:867-969 with live Qhull: (dist, winning index, Fv triple, plane normal,
    facet count, Qhull text for injection)."""
    rounded = np.array([[float(f"{v:g}") for v in p] for p in pts_full])     # ostream << (6 digits)
    planes, fv, ntext, vtext = qhull_lib.qconvex(rounded)                    # parsed as >> reads them
    first = np.array([f[0] for f in fv])
    best, dist = 0, None
    for i in range(len(fv)):
        P = pts_full[first[i]]
        t = abs(planes[i, 0] * (vrel[0] - P[0]) + planes[i, 1] * (vrel[1] - P[1]) + planes[i, 2] * (vrel[2] - P[2]))
        if dist is None or t < dist:
            dist, best = t, i
    return dist, best, list(fv[best]) + [-1] * max(0, 3 - len(fv[best])), planes[best, :3].copy(), len(fv), \
        (rounded, fv, planes)


def workload(name, N, H, box, seed, g, inject=None):
    x, vg = lqro.synthetic_swarm(N, box=box, seed=seed) if box else lqro.synthetic_swarm(N)
    T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = pyoracle.sphere(100)
    pyoracle.set_hull_rule(0)
    _, recs = pyoracle.step(T, NCF, S, x, vg, threads=8)
    carry = np.zeros(3)                     # normalVector (LQRO:1385)
    pairs, planes_row, merged = [], {}, []
    for r in recs:                          # (i, j) order: the reference's loop
        if not (r["flags"] & 1):
            continue                        # n <= 4: normalVector untouched (LQRO:1409)
        i, j = int(r["i"]), int(r["j"])
        if not (r["flags"] & 2):
            carry = r["normal"].copy()      # run_gjk wrote it (LQRO:850-852)
            continue
        _, _, pts = pyoracle.pair(T, NCF, S, x[i], x[j], i, j, want_points=True)
        vrel = x[i, 3:6] - x[j, 3:6]
        dist, best, fvb, nrm, nf, q = reference_hull(pts, vrel)
        nonsimp = [k for k, f in enumerate(q[1]) if len(f) != 3]
        if nonsimp:   # Qhull merged facets here (its default pre-merge)
            merged.append((i, j, nf, len(nonsimp), int(best in nonsimp),
                           [(list(q[1][k]), q[2][k].copy()) for k in nonsimp]))
        fvb = fvb[:3]
        stale = best == 0
        if not stale:
            carry = nrm
        pairs.append((i, j, int(r["n_reach"]), nf, best, *fvb, dist, *carry, int(stale)))
        planes_row[(i, j)] = (dist, carry.copy())
        if inject is not None and len(inject) < 6 and nf < 700:
            inject.append((pts, q, vrel, dist, best, carry.copy(), stale))
    newv = np.zeros((N, 3))
    for i in range(N):
        pl = []
        for r in recs[recs["i"] == i]:
            if not (r["flags"] & 1):
                continue
            j = int(r["j"])
            if (i, j) in planes_row:
                d, n = planes_row[(i, j)]
                d *= 0.5                                                # LQRO:1416
                p = np.array([x[i, 3] + 1.0 * d * n[0], x[i, 4] + 1.0 * d * n[1], x[i, 5] + 1.0 * d * n[2],
                              n[0], n[1], n[2]], np.float64).astype(np.float32)   # LQRO:1208-1221
            else:
                p = np.concatenate([r["plane_point"], r["plane_normal"]]).astype(np.float32)
            pl.append(p)
        newv[i] = pyoracle.newv(np.array(pl, np.float32).reshape(-1, 6), vg[i])
    dt = np.dtype([("i", "<i4"), ("j", "<i4"), ("n_reach", "<i4"), ("n_facets", "<i4"), ("best", "<i4"),
                   ("fv", "<i4", (3,)), ("dist", "<f8"), ("normal", "<f8", (3,)), ("stale", "<i4")])
    arr = np.zeros(len(pairs), dt)
    for k, p in enumerate(pairs):
        arr[k] = (p[0], p[1], p[2], p[3], p[4], p[5:8], p[8], p[9:12], p[12])
    mdt = np.dtype([("i", "<i4"), ("j", "<i4"), ("n_facets", "<i4"), ("n_merged", "<i4"), ("winner_merged", "<i4")])
    marr = np.zeros(len(merged), mdt)
    mfac, moffs, mplanes, mpoffs = [], [0], [], [0]
    for k, (i, j, nf, nm, wm, facets) in enumerate(merged):
        marr[k] = (i, j, nf, nm, wm)
        for f, pl in facets:
            mfac.extend(int(v) for v in f)
            moffs.append(len(mfac))
            mplanes.append(pl)
        mpoffs.append(len(mplanes))
    mout = dict(merged=marr, merged_facets=np.array(mfac, np.int32), merged_offs=np.array(moffs, np.int64),
                merged_planes=np.array(mplanes, np.float64).reshape(-1, 4), merged_pairoffs=np.array(mpoffs, np.int64))
    return x, vg, arr, newv, carry, mout


def main():
    g = pyoracle.synthesize()
    summary, out = {}, {}
    inject = []
    for name, N, H, box, seed in WORKLOADS:
        t0 = time.time()
        x, vg, arr, newv, carry, mout = workload(name, N, H, box, seed, g, inject if name == "dense" else None)
        for k, v in mout.items():
            out[f"{name}_{k}"] = v
        out[f"{name}_pairs"] = arr
        out[f"{name}_newv"] = newv
        out[f"{name}_carry"] = carry
        # the oracle's Qhull-order rule on the same step (planes read back as printed)
        T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
        S = pyoracle.sphere(100)
        pyoracle.set_hull_rule(1, round16=True)
        pyoracle.carry_normal(np.zeros(3))
        xo, vo = (lqro.synthetic_swarm(N, box=box, seed=seed) if box else lqro.synthetic_swarm(N))
        v1, r1 = pyoracle.step(T, NCF, S, xo, vo, threads=8)
        pyoracle.set_hull_rule(0)
        ins = r1[(r1["flags"] & 2) != 0]
        same = sum(int(a["dist"] == b["dist"] and np.array_equal(a["normal"], b["normal"])
                       and np.array_equal(a["facet"], b["fv"])) for a, b in zip(ins, arr))
        summary[name] = dict(
            inside_pairs=len(arr), stale_pairs=int(arr["stale"].sum()),
            qhull_merge_pairs=int(((ins["flags"] & 0x80) != 0).sum()),
            qconvex_merged_pairs=len(mout["merged"]),
            qconvex_merged_winners=int(mout["merged"]["winner_merged"].sum()),
            oracle_pairs_bit_exact=same, oracle_rows_newv_bit_exact=int((v1 == newv).all(1).sum()),
            rows=N, seconds=round(time.time() - t0, 1))
        print(name, summary[name], flush=True)
    for k, (pts, (rounded, fv, planes), vrel, dist, best, nrm, stale) in enumerate(inject):
        out[f"inject{k}_pts"] = pts
        out[f"inject{k}_rounded"] = rounded
        out[f"inject{k}_fv"] = np.array(fv, np.int32)
        out[f"inject{k}_planes"] = planes
        out[f"inject{k}_vrel"] = vrel
        out[f"inject{k}_expect"] = np.array([dist, best, int(stale), *nrm])
    np.savez_compressed(os.path.join(HERE, "qhull_order.npz"), **out)
    s = json.dumps(summary, indent=1)
    print(s)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(s)


if __name__ == "__main__":
    main()
