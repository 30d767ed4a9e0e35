"""The inside-hull branch against the reference's own selection rule
(LQRObstacles.cpp:867-969), quantified (tests/golden/hull_rule.npz, made by
make_golden_hull_rule.py with scipy's Qhull standing in for qconvex.exe —
Qhull reproduces the reference's own pointList/Planes/facetVertices fixture
facet for facet, in order, first vertices included).

Pinned here:
  * the hull: this build's facet set equals Qhull's on every inside pair of
    the dense swarm (92) and the C3 bench swarm (177);
  * the oracle's (hence the GPU's) hull-branch distance is the fixture's;
  * the measured gap to the reference's rule (first Fv vertex, Qhull facet
    order, stale normal when facet 0 wins): distance within 1e-4 absolute
    (6-significant-digit rounding of the hull input, SURVEY §7 hazard 1)
    on every pair; same normal on every pair whose arg-min facet agrees.
The canonical rule (the default without LQRO_FLAG_QHULL_ORDER) is a
DEVIATION, not parity: test_canonical_rule_is_not_parity fails if its newV
were reported as the reference's.  The reference's own rule — Qhull's build
order restated (oracle/lqro_qhull.c, k_qhull) — is pinned bit for bit in
tests/test_qhull_order.py and tests/test_gpu_qhull_order.py."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIX = os.path.join(GOLDEN, "hull_rule.npz")


def test_hull_facet_sets_equal_qhull():
    d = np.load(FIX)
    for w in ("dense", "c3"):
        assert len(d[f"{w}_facets_equal"]) > 50
        assert d[f"{w}_facets_equal"].all(), w


def test_gap_to_reference_rule_is_bounded():
    d = np.load(FIX)
    for w in ("dense", "c3"):
        dd = np.abs(d[f"{w}_dist_ours"] - d[f"{w}_dist_ref"])
        assert dd.max() <= 1e-4, (w, dd.max())
        same = np.abs(d[f"{w}_normal_ours"] - d[f"{w}_normal_ref"]).max(axis=1) <= 1e-9
        stale = d[f"{w}_stale"]
        # the normals differ only where the reference kept a stale normal or
        # picked another facet through its first-vertex distance
        assert (~same & ~stale).sum() <= 0.05 * len(same), w


def test_oracle_reproduces_fixture_distances(oracle, lqro_mod, gains):
    d = np.load(FIX)
    x, vg = lqro_mod.synthetic_swarm(32, box=3.0, seed=11)
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], 45)
    _, recs = oracle.step(T, NCF, oracle.sphere(100), x, vg, threads=4)
    inside = recs[(recs["flags"] & 2) != 0]
    assert np.array_equal(inside["i"], d["dense_i"]) and np.array_equal(inside["j"], d["dense_j"])
    assert np.array_equal(inside["dist"].view(np.uint64), d["dense_dist_ours"].view(np.uint64))


def test_reference_rule_live_with_qhull(oracle, lqro_mod, gains):
    """Where scipy is importable, re-derive the reference rule for a few dense
    pairs and match the fixture (checks the generator, not the build)."""
    pytest.importorskip("scipy.spatial")
    import sys
    sys.path.insert(0, GOLDEN)
    from make_golden_hull_rule import reference_rule
    d = np.load(FIX)
    x, _ = lqro_mod.synthetic_swarm(32, box=3.0, seed=11)
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], 45)
    S = oracle.sphere(100)
    for k in range(0, len(d["dense_i"]), 23):
        if d["dense_stale"][k]:
            continue
        i, j = int(d["dense_i"][k]), int(d["dense_j"][k])
        _, _, pts = oracle.pair(T, NCF, S, x[i], x[j], i, j, want_points=True)
        dist, nrm, _, _ = reference_rule(pts, x[i, 3:6] - x[j, 3:6])
        assert dist == d["dense_dist_ref"][k]
        assert np.array_equal(nrm, d["dense_normal_ref"][k])


def test_canonical_rule_is_not_parity():
    """The canonical rule's newV (hull_rule.npz) against the reference loop
    over live Qhull (qhull_order.npz): rows with a hull pair differ beyond
    1e-5 — the canonical rule must not be reported as reference parity; the
    Qhull-order rule (LQRO_FLAG_QHULL_ORDER) is."""
    a = np.load(FIX)
    b = np.load(os.path.join(GOLDEN, "qhull_order.npz"))
    for w, need in (("dense", 1), ("c3", 1)):
        rows = a[f"{w}_rows"]
        ref = b[f"{w}_newv"][rows]
        ours = a[f"{w}_newv_ours"]
        rel = np.abs(ours - ref).max(1) / np.maximum(np.abs(ref).max(1), 1e-30)
        assert (rel > 1e-5).sum() >= need, w
