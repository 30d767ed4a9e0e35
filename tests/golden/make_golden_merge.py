#!/usr/bin/env python3
"""Hulls whose winning facet qconvex MERGES.  TEST INFRASTRUCTURE, build
container only (live Qhull through qhull_lib, scipy's qhull_r 2019.1).

qconvex's default pre-merge (C-0) joins coplanar and non-convex facets, and
convexHull (LQRObstacles.cpp:925-968) then measures a merged facet from the
first vertex of its Fv list with its merged plane.  This build's k_qhull
restates Qhull's build merge-free: where Qhull's merge tests fire it flags
the pair LQRO_REC_QHMERGE, and where the winner may be a merged facet also
LQRO_REC_QHMERGE_WIN (include/lqro.h) — the pair's facet, distance and
normal are then not the reference's.  These cases are inputs where qconvex's
winner IS a merged facet, so the flag must fire.

Cases (points before the 6-digit rounding convexHull prints, LQRO:869-874):
  cube_top / cube_side: random points on the six faces of a cube (each face
      exactly coplanar), vrel near a face: qconvex's winner is the merged face;
  capped: an ellipsoid cloud whose top is flattened onto a plane (a coplanar
      cap), vrel just below the cap.
Stores tests/golden/qhull_merge.npz: per case <c>_pts (full), <c>_rounded,
<c>_vrel, and qconvex's side: <c>_fv (Fv lists flattened, <c>_fvoff
offsets), <c>_planes (as printed and read back), <c>_expect = [winner index,
winner merged (Fv list longer than 3), dist, stale, normal xyz].

Usage:  python tests/golden/make_golden_merge.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(ROOT, "oracle")]
import pyoracle  # noqa: E402  (round6 only: the %g rounding of LQRO:871-873)
import qhull_lib  # noqa: E402


def cube(rng, n_per_face=40, s=2.0, c=(3.0, -1.0, 2.0)):
    pts = []
    for ax in range(3):
        for sg in (-1, 1):
            u = rng.uniform(-1, 1, (n_per_face, 2))
            p = np.zeros((n_per_face, 3))
            p[:, ax] = sg
            o = [a for a in range(3) if a != ax]
            p[:, o[0]], p[:, o[1]] = u[:, 0], u[:, 1]
            pts.append(p)
    return np.concatenate(pts) * s + np.array(c)


def capped(rng, n=600, cap=0.6):
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    p = u * np.array([1.5, 1.0, 0.8]) + np.array([-2.0, 4.0, 1.0])
    top = 1.0 + 0.8 * cap
    p[:, 2] = np.minimum(p[:, 2], top)
    return p


def reference_rule(full, planes, fv, vrel):
    """LQRO:955-968 over qconvex's output: first Fv vertex at full precision,
    planes as read back, strict '<'; facet 0 keeps the carried normal."""
    best, d = 0, None
    nrm = None
    for f, (pl, verts) in enumerate(zip(planes, fv)):
        P = full[verts[0]]
        t = abs(pl[0] * (vrel[0] - P[0]) + pl[1] * (vrel[1] - P[1]) + pl[2] * (vrel[2] - P[2]))
        if d is None or t < d:
            d, best = t, f
            if f > 0:
                nrm = pl[:3].copy()
    return best, d, best == 0, (nrm if nrm is not None else np.zeros(3))


def main():
    rng = np.random.default_rng(20261018)
    cases = {}
    c = cube(rng)
    cases["cube_top"] = (c, np.array([3.0, -1.0, 2.0]) + np.array([0.1, 0.2, 1.9]))
    cases["cube_side"] = (c, np.array([3.0, -1.0, 2.0]) + np.array([-1.85, 0.3, -0.2]))
    p = capped(rng)
    cases["capped"] = (p, np.array([-2.0, 4.0, 1.0]) + np.array([0.05, -0.1, 0.8 * 0.6 - 0.02]))
    out = {}
    for name, (full, vrel) in cases.items():
        rounded = np.array([[pyoracle.round6(v) for v in row] for row in full])
        planes, fv, _, _ = qhull_lib.qconvex(rounded)
        best, d, stale, nrm = reference_rule(full, planes, fv, vrel)
        merged = len(fv[best]) > 3
        out[f"{name}_pts"] = full
        out[f"{name}_rounded"] = rounded
        out[f"{name}_vrel"] = vrel
        out[f"{name}_fv"] = np.array([v for f in fv for v in f], np.int32)
        out[f"{name}_fvoff"] = np.cumsum([0] + [len(f) for f in fv]).astype(np.int32)
        out[f"{name}_planes"] = planes
        out[f"{name}_expect"] = np.array([best, int(merged), d, int(stale), *nrm])
        print(name, "facets", len(fv), "merged facets", sum(len(f) > 3 for f in fv), "winner", best,
              "merged" if merged else "simplicial", "dist", d, flush=True)
    np.savez_compressed(os.path.join(HERE, "qhull_merge.npz"), **out)


if __name__ == "__main__":
    main()
