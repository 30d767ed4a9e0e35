"""k_qhull (LQRO_FLAG_QHULL_ORDER): the inside-hull branch with the
reference's own rule — Qhull's facet order, each facet's first Fv vertex,
strict '<', the loop-carried normalVector when facet 0 wins
(LQRObstacles.cpp:925-968, 1385) — against

- the oracle's restatement of Qhull's build (oracle/lqro_qhull.c, pinned to
  live Qhull in tests/test_qhull_order.py), bit for bit: records (facet in
  Fv order, distance, normal, flags, half-plane) and new velocities;
- tests/golden/qhull_order.npz, the reference's pair loop over live Qhull
  (planes read back as qconvex prints them, %.16g — the GPU reads them back
  the same way, lqro_dec16.hpp): the same facets, distances, normals and
  every row's newV, bit for bit."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

QO = os.path.join(GOLDEN, "qhull_order.npz")


def _golden():
    return np.load(QO)


def test_qhull_hook_on_injected_pairs(lqro_mod, oracle, gains):
    """Qhull's full output for six dense-swarm pairs: k_qhull's build and
    selection through the test hook equal the oracle's and the golden's."""
    d = _golden()
    ctx = lqro_mod.Context(lqro_mod.config(2, 45, 100))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    oracle.set_hull_rule(1, round16=True)
    try:
        for k in range(6):
            pts, rounded, fv = d[f"inject{k}_pts"], d[f"inject{k}_rounded"], d[f"inject{k}_fv"]
            vrel = d[f"inject{k}_vrel"]
            dist_g, best_g, stale_g = d[f"inject{k}_expect"][:3]
            rec, st, fl = ctx.debug_qhull(rounded, pts, vrel, max_facets=4096)
            n_same = 0
            while n_same < min(len(fl), len(fv)) and np.array_equal(fl[n_same], fv[n_same]):
                n_same += 1
            assert st == 0 and len(fl) == len(fv) and n_same == len(fv), \
                f"pair {k}: status {st}, {len(fl)} facets ({len(fv)} in Qhull), first difference at {n_same}"
            nf, dist_o, nrm_o, fac_o, qst = oracle.hull_branch_ref(pts, vrel)
            assert rec["n_facets"] == nf == fv.shape[0]
            assert list(rec["facet"]) == list(fac_o) == list(fv[int(best_g)])
            assert rec["dist"] == dist_o
            assert bool(rec["flags"] & lqro_mod.REC_STALE) == (nrm_o is None) == bool(stale_g)
            if nrm_o is not None:
                assert np.array_equal(rec["normal"], nrm_o)
            assert rec["dist"] == dist_g, (k, rec["dist"], dist_g)   # the planes read back at 16 digits
    finally:
        oracle.set_hull_rule(0)
        ctx.close()


def test_qhull_hook_on_reference_fixture(lqro_mod, oracle, gains):
    """k_qhull on the reference's own Qhull fixture (tests/golden/qhull:
    pointList.txt, the qconvex input LQRO:869-880 writes): the facet list in
    the order of facetVertices.txt (qconvex Fv) with every facet's vertices
    in Fv order, and for relative velocities inside the hull the selection
    of LQRO:925-968 (first Fv vertex, strict '<', facet 0 keeps the carried
    normal) equal to the oracle's, bit for bit."""
    from test_oracle_golden import _qhull_fixture
    pts, planes, fv = _qhull_fixture()
    pts = np.ascontiguousarray(pts, np.float64)
    ctx = lqro_mod.Context(lqro_mod.config(2, 100, 100))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    oracle.set_hull_rule(1, round16=True)
    try:
        cen = pts.mean(0)
        for k in (None, 0, 100, 517, 1000):
            vrel = cen if k is None else cen + 0.9 * (pts[k] - cen)
            rec, st, fl = ctx.debug_qhull(pts, pts, vrel, max_facets=4096)
            assert st == 0
            assert [list(map(int, r)) for r in fl] == [f[1:] for f in fv]
            nf, dist_o, nrm_o, fac_o, _ = oracle.hull_branch_ref(pts, vrel)
            assert rec["n_facets"] == nf == len(fv)
            assert list(rec["facet"]) == list(fac_o)
            assert rec["dist"] == dist_o
            assert bool(rec["flags"] & lqro_mod.REC_STALE) == (nrm_o is None)
            if nrm_o is not None:
                assert np.array_equal(rec["normal"], nrm_o)
    finally:
        oracle.set_hull_rule(0)
        ctx.close()


def _ref_step(lqro_mod, oracle, gains, N, H, box, seed, steps=1):
    kw = {} if box is None else dict(box=box, seed=seed)
    x, vg = lqro_mod.synthetic_swarm(N, **kw)
    ctx = lqro_mod.Context(lqro_mod.config(N, H, 100, flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    out = []
    for _ in range(steps):
        v = ctx.step(x, vg)
        out.append((v, ctx.records(), ctx.stats(), ctx.carry_normal()))
    ctx.close()
    return x, vg, out


@pytest.mark.parametrize("case", ["dense", "c2"])
def test_qhull_order_step_vs_oracle(lqro_mod, oracle, gains, case):
    N, H, box, seed = (32, 45, 3.0, 11) if case == "dense" else (64, 50, None, None)
    x, vg, out = _ref_step(lqro_mod, oracle, gains, N, H, box, seed, steps=2)
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    S = oracle.sphere(100)
    oracle.set_hull_rule(1, round16=True)
    oracle.carry_normal(np.zeros(3))
    try:
        for v, r, st, carry in out:
            rv, rr = oracle.step(T, NCF, S, x, vg, threads=8)
            assert st["hull_fail"] == 0
            for f in ("n_reach", "flags", "facet", "n_facets", "dist", "normal", "plane_point", "plane_normal"):
                a, b = r[f], rr[f]
                if f == "flags":
                    a, b = a & ~lqro_mod.REC_LOCAL, b
                assert np.array_equal(a, b), f
            assert np.array_equal(v.view(np.uint64), rv.view(np.uint64))
            assert np.array_equal(carry, oracle.carry_normal())
    finally:
        oracle.set_hull_rule(0)


@pytest.mark.parametrize("case", ["dense", "c2", "c3", "crowd22"])
def test_qhull_order_vs_reference_loop(lqro_mod, oracle, gains, case):
    """The reference's pair loop over live Qhull (golden): every inside pair's
    facet, distance and (carried) normal; every row's newV within 1e-5."""
    d = _golden()
    N, H, box, seed = {"dense": (32, 45, 3.0, 11), "c2": (64, 50, None, None),
                       "c3": (1024, 100, None, None), "crowd22": (1024, 100, 22.0, 7)}[case]
    x, vg, out = _ref_step(lqro_mod, oracle, gains, N, H, box, seed)
    v, r, st, _ = out[0]
    g = d[f"{case}_pairs"]
    ins = r[(r["flags"] & lqro_mod.REC_INSIDE) != 0]
    bad = ins[(ins["flags"] & lqro_mod.REC_HULLFAIL) != 0]
    assert len(ins) == len(g) and st["hull_fail"] == 0, \
        [(int(b["i"]), int(b["j"]), int(b["n_reach"]), -int(b["n_facets"]) - 1) for b in bad]
    assert np.array_equal(ins["i"], g["i"]) and np.array_equal(ins["j"], g["j"])
    assert np.array_equal(ins["facet"], g["fv"])
    # Qhull's default pre-merge: the pairs whose qconvex output holds merged
    # (non-simplicial) facets are stored with those facets (<w>_merged*).
    # k_qhull builds merge-free and flags every pair where Qhull's merge tests
    # fire (REC_QHMERGE): each qconvex-merged pair must be flagged, its winner
    # must be a simplicial facet (the selection above then equals Qhull's), and
    # every other pair's facet count equals qconvex's
    qm = d[f"{case}_merged"]
    flagged = {(int(a), int(b)) for a, b, f in zip(ins["i"], ins["j"], ins["flags"]) if f & lqro_mod.REC_QHMERGE}
    qmerged = {(int(a), int(b)) for a, b in zip(qm["i"], qm["j"])}
    assert qmerged <= flagged, sorted(qmerged - flagged)
    assert not qm["winner_merged"].any(), qm[qm["winner_merged"] != 0]
    keep = np.array([(int(a), int(b)) not in qmerged for a, b in zip(ins["i"], ins["j"])], bool)
    assert np.array_equal(ins["n_facets"][keep], g["n_facets"][keep])
    assert np.array_equal((ins["flags"] & lqro_mod.REC_STALE) != 0, g["stale"] != 0)
    # the planes as convexHull reads them back (16 digits, LQRO:889-899): the
    # reference loop's distances, normals and new velocities, bit for bit
    bad_d = np.nonzero(ins["dist"].view(np.uint64) != g["dist"].view(np.uint64))[0]
    assert len(bad_d) == 0, [(int(ins["i"][k]), int(ins["j"][k]), ins["dist"][k], g["dist"][k]) for k in bad_d[:5]]
    assert np.array_equal(ins["normal"].view(np.uint64), g["normal"].view(np.uint64))
    gv = d[f"{case}_newv"]
    bad_v = np.nonzero((v.view(np.uint64) != gv.view(np.uint64)).any(1))[0]
    assert len(bad_v) == 0, f"rows whose newV differs from the reference loop's: {bad_v[:10]}"
