#!/usr/bin/env python3
"""Golden fixture for GJK's backup procedure (gjk.cpp:663-706), from the
REFERENCE's own code.  TEST INFRASTRUCTURE, build container only.

The backup runs when the default sub-algorithm finds no valid subset; on the
synthetic C3 swarm that is about 2 pairs in 10^6.  This script finds such
pairs with the oracle on full C3 steps (two seeds), then runs the
reference's pair body on them (oracle/_ref/libref.so ref_pair = LQRO:1397-1418
with the reference's findFG, createObstacle, findReachableObstacle,
pointInHull / run_gjk and createHalfPlanes; ref_gjk = gjk_distance) and
stores inputs and outputs in tests/golden/gjk_backup.npz.

Usage:  python tests/golden/make_golden_backup.py
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "lqr-obstacles_amd")]
import pyoracle  # noqa: E402
import lqro  # noqa: E402  (the pure-Python swarm generator only)

N, H, NP = 1024, 100, 100


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def main():
    ref = pyoracle.reflib()
    assert ref is not None, "needs oracle/_ref/libref.so"
    ref.ref_gjk.restype = C.c_double
    g = pyoracle.synthesize()
    T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = pyoracle.sphere(NP)
    rows = []
    for seed in (lqro.SEED, 0x5EED):
        x, vg = lqro.synthetic_swarm(N, seed=seed)
        _, recs = pyoracle.step(T, NCF, S, x, vg, threads=8)
        for r in recs[(recs["flags"] & 4) != 0]:
            rows.append((x[r["i"]].copy(), x[r["j"]].copy()))
    print(f"{len(rows)} backup pairs")
    out = {k: [] for k in ("xi", "xj", "status", "n_reach", "dist", "normal", "plane", "gjk_sqd",
                           "gjk_wpt_vrel", "gjk_wpt_hull")}
    idx = np.zeros(H * NP, np.int32)
    pts = np.zeros((H * NP, 3))
    for xi, xj in rows:
        n = C.c_int(0)
        dist = np.zeros(1)
        nrm, wv, wh = np.zeros(3), np.zeros(3), np.zeros(3)
        pl = np.zeros(6, np.float32)
        st = ref.ref_pair(NP, H, 4, C.c_double(30.0), _p(g["A"]), _p(g["B"]), _p(g["L"]), _p(g["E"]),
                          _p(xi), _p(xj), C.byref(n), _p(idx), _p(pts), _p(dist), _p(nrm), _p(wv), _p(wh),
                          _p(pl))
        vrel = np.ascontiguousarray(xi[3:6] - xj[3:6])
        w1, w2 = np.zeros(3), np.zeros(3)
        sq = ref.ref_gjk(n.value, _p(pts), _p(vrel), _p(w1), _p(w2))
        for k, v in (("xi", xi), ("xj", xj), ("status", st), ("n_reach", n.value), ("dist", dist[0]),
                     ("normal", nrm), ("plane", pl), ("gjk_sqd", sq), ("gjk_wpt_vrel", w1),
                     ("gjk_wpt_hull", w2)):
            out[k].append(v)
    np.savez_compressed(os.path.join(HERE, "gjk_backup.npz"), H=H, NP=NP,
                        **{k: np.array(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
