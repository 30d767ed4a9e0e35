"""The oracle pinned against the reference's own outputs (CPU, no GPU).

tests/golden/*.npz were produced by tests/golden/make_golden.py from the
reference's functions compiled in this container (oracle/_ref/libref.so);
tests/golden/qhull/ is the reference's own Qhull triple.  Bar: integer
outputs and every fp64/fp32 value bit-exact — the oracle follows the
reference's operation order (hoisting F_k, G_k per agent changes no bits).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def _same_bits(a, b):
    a, b = np.atleast_1d(np.asarray(a)), np.atleast_1d(np.asarray(b))
    return a.shape == b.shape and a.dtype == b.dtype and \
        np.array_equal(a.view(np.uint8), b.view(np.uint8))


def test_gains_bit_exact(oracle):
    """controlMatrices (LQRO:520-582): A, B, c, L, E, Lh, Eh."""
    ref = _load("gains.npz")
    got = oracle.synthesize()
    for k in ("A", "B", "c", "L", "E", "Lh", "Eh"):
        assert _same_bits(got[k], ref[k]), k


@pytest.mark.parametrize("np_", [100, 50])
def test_sphere_bit_exact(oracle, np_):
    """createSpheres (LQRO:735-750)."""
    ref = _load("gains.npz")[f"sphere{np_}"]
    assert _same_bits(oracle.sphere(np_), ref)


@pytest.mark.parametrize("scenario", ["swap", "c2", "dense"])
def test_pairs_bit_exact(oracle, scenario):
    """createObstacle + findReachableObstacle + run_gjk + createHalfPlanes
    (LQRO:1401-1417) pair by pair."""
    g = _load("gains.npz")
    P = _load("pairs.npz")
    H = 50
    T, NCF = oracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = oracle.sphere(100)
    x = P[f"{scenario}_x"]
    n_inside = 0
    for k in range(P[f"{scenario}_i"].size):
        i, j = int(P[f"{scenario}_i"][k]), int(P[f"{scenario}_j"][k])
        rec, idx, _ = oracle.pair(T, NCF, S, x[i], x[j], i, j, want_points=True)
        status = int(P[f"{scenario}_status"][k])
        n = int(P[f"{scenario}_n_reach"][k])
        assert rec["n_reach"] == n, (i, j)
        assert np.uint64(rec["reach_hash"]) == P[f"{scenario}_reach_hash"][k], (i, j)
        head = P[f"{scenario}_head"][k]
        tail = P[f"{scenario}_tail"][k]
        assert np.array_equal(idx[:16], head[:min(16, n)])
        if n:
            assert np.array_equal(idx[-16:], tail[:min(16, n)])
        gated = not (n > 4)
        assert bool(rec["flags"] & 1) == (not gated)
        assert bool(rec["flags"] & 2) == (status == 1), (i, j)
        if status == 1:
            n_inside += 1
            # the reference's GJK witnesses of the inside pair (before convexHull)
            assert _same_bits(rec["wpt_vrel"], P[f"{scenario}_wpt_vrel"][k])
            assert _same_bits(rec["wpt_hull"], P[f"{scenario}_wpt_hull"][k])
            continue
        if status == 2:
            continue
        assert _same_bits(rec["dist"], P[f"{scenario}_dist"][k]), (i, j)
        assert _same_bits(rec["normal"], P[f"{scenario}_normal"][k]), (i, j)
        assert _same_bits(rec["wpt_vrel"], P[f"{scenario}_wpt_vrel"][k])
        assert _same_bits(rec["wpt_hull"], P[f"{scenario}_wpt_hull"][k])
        pl = np.concatenate([rec["plane_point"], rec["plane_normal"]]).astype(np.float32)
        assert _same_bits(pl, P[f"{scenario}_plane"][k]), (i, j)
    if scenario == "dense":
        assert n_inside > 0


def test_newv_bit_exact(oracle):
    """calculateNewV → linearProgram3/4 (LQRO:1001-1234), fp32."""
    d = _load("newv.npz")
    offs = d["offsets"]
    for k in range(d["newv"].shape[0]):
        pl = d["planes"][offs[k]:offs[k + 1]]
        got = oracle.newv(pl, d["vgoal"][k])
        assert _same_bits(got, d["newv"][k]), k


def test_newv_c3_hardest_rows(oracle):
    """The C3 rows whose LP runs linearProgram4 longest (lp_rows.npz, checked
    against the reference's calculateNewV when made): the oracle bit for bit."""
    d = _load("lp_rows.npz")
    for k in range(d["newv"].shape[0]):
        got = oracle.newv(d["planes"][k], d["vgoal"][k], float(d["vmax_lp"]))
        assert _same_bits(got, d["newv"][k]), k
        assert oracle.lp_chain(d["planes"][k], d["vgoal"][k], float(d["vmax_lp"])) == d["chain"][k]


@pytest.mark.parametrize("scenario", ["c2", "swap"])
def test_row_newv_bit_exact(oracle, scenario):
    """The whole row body (LQRO:1393-1435) for the golden rows."""
    g = _load("gains.npz")
    d = _load("steps.npz")
    x, vg, rows = d[f"{scenario}_x"], d[f"{scenario}_vgoal"], d[f"{scenario}_rows"]
    T, NCF = oracle.tables(g["A"], g["B"], g["L"], g["E"], 50)
    S = oracle.sphere(100)
    r0, r1 = int(rows[0]), int(rows[-1]) + 1
    newv, _ = oracle.step(T, NCF, S, x, vg, rows=(r0, r1), records=False)
    for i in rows:
        if d[f"{scenario}_ok"][i]:
            assert _same_bits(newv[i], d[f"{scenario}_newv"][i]), i


def test_reference_accumulates_planes(oracle):
    """Rows 0..3 of C2 through the reference's driver in ONE call equal the
    per-row results: calculateNewV empties orcaPlanes_ after each row's LP
    (LQRO:1233), so no plane carries over to the next row."""
    d = _load("steps.npz")
    acc = d["c2_accum_newv"]
    per = d["c2_newv"]
    for i in range(4):
        assert _same_bits(acc[i], per[i]), i


@pytest.mark.parametrize("scenario", ["swap", "c2", "dense"])
def test_reference_driver_one_call(oracle, scenario):
    """The whole pair loop (LQRO:1391-1436) of the reference over all rows in
    one call (tests/golden/driver.npz: its loop-carried distance /
    normalVector / insideHull and per-row orcaPlanes_), against the oracle's
    step: every row without an inside-hull pair bit for bit (the reference
    harness stops inside pairs before qconvex.exe)."""
    d = _load("driver.npz")
    g = oracle.synthesize()
    H = int(d[f"{scenario}_H"])
    x, vg = d[f"{scenario}_x"], d[f"{scenario}_vgoal"]
    T, NCF = oracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    newv, _ = oracle.step(T, NCF, oracle.sphere(100), x, vg, records=False, threads=4)
    ok = d[f"{scenario}_ok"].astype(bool)
    assert ok.sum() >= {"swap": 4, "c2": 62, "dense": 2}[scenario]
    assert np.array_equal(newv[ok].view(np.uint64), d[f"{scenario}_newv"][ok].view(np.uint64))


def _qhull_fixture():
    q = os.path.join(GOLDEN, "qhull")
    with open(os.path.join(q, "pointList.txt")) as f:
        dim = int(f.readline())
        n = int(f.readline())
        pts = np.array([[float(v) for v in f.readline().split()] for _ in range(n)])
    assert dim == 3
    with open(os.path.join(q, "Planes.txt")) as f:
        assert int(f.readline()) == 4
        m = int(f.readline())
        planes = np.array([[float(v) for v in f.readline().split()] for _ in range(m)])
    with open(os.path.join(q, "facetVertices.txt")) as f:
        m2 = int(f.readline())
        fv = [[int(v) for v in f.readline().split()] for _ in range(m2)]
    assert m == m2
    return pts, planes, fv


def test_hull_matches_reference_qhull_fixture(oracle):
    """The hull of the reference's pointList.txt (qconvex input, already
    %g-rounded) has exactly the facets of its facetVertices.txt, and every
    facet plane matches Planes.txt (qconvex "n" output, %.16g)."""
    pts, planes, fv = _qhull_fixture()
    got = oracle.hull(pts)
    ref = sorted(tuple(sorted(f[1:])) for f in fv)
    assert all(f[0] == 3 for f in fv)
    assert sorted(tuple(sorted(int(v) for v in t)) for t in got) == ref
    # planes: outward unit normal n and offset o with n.x + o = 0 on the facet
    for f, pl in zip(fv, planes):
        a, b, c = pts[f[1]], pts[f[2]], pts[f[3]]
        nrm = np.cross(b - a, c - a)
        nrm /= np.linalg.norm(nrm)
        if np.dot(nrm, pl[:3]) < 0:
            nrm = -nrm
        assert np.allclose(nrm, pl[:3], atol=1e-9)
        assert abs(np.dot(pl[:3], a) + pl[3]) < 1e-9 * (1 + abs(pl[3]))


def test_qhull_order_matches_reference_fixture_in_order(oracle):
    """The oracle's restatement of Qhull's build (oracle/lqro_qhull.c) on the
    reference's pointList.txt reproduces qconvex's own output IN ORDER: the
    facet list of facetVertices.txt (qconvex Fv, LQRO:880) facet for facet,
    each facet's vertex list in Fv order (its first vertex is the one
    LQRO:925-937 measures the distance from), and the planes of Planes.txt
    (qconvex n, LQRO:879, printed %.16g) to 1e-15 relative."""
    pts, planes, fv = _qhull_fixture()
    st, got, pl, _ = oracle.qhull(np.ascontiguousarray(pts, np.float64))
    assert st == 0, f"build status {st}"
    assert got.shape == (len(fv), 3)
    assert [list(map(int, r)) for r in got] == [f[1:] for f in fv]
    err = np.abs(pl - planes) / np.maximum(np.abs(planes), 1.0)
    assert err.max() <= 1e-15, err.max()


def test_hull_cases_are_closed_and_convex(oracle):
    """The inside-hull pairs of the dense golden set (whose qconvex step the
    reference cannot run here): the oracle's hull of the %g-rounded points is
    a closed 2-manifold with every point on the inner side of every facet.
    Facet identity beyond the Qhull fixture is 'parity unpinned'."""
    P = _load("pairs.npz")
    assert int(P["n_hull"]) > 0
    for h in range(int(P["n_hull"])):
        full = P[f"hull{h}_pts"]
        pts = np.vectorize(oracle.round6)(full)
        F = oracle.hull(pts)
        edges = {}
        for t in F:
            for a, b in ((t[0], t[1]), (t[1], t[2]), (t[2], t[0])):
                e = (min(a, b), max(a, b))
                edges[e] = edges.get(e, 0) + 1
        assert all(v == 2 for v in edges.values())
        assert len(F) == 2 * len(set(F.ravel())) - 4          # Euler, triangulated
        cen = pts[np.unique(F)].mean(0)
        scale = np.abs(pts).max() + 1
        for t in F:
            a, b, c = pts[t[0]], pts[t[1]], pts[t[2]]
            nrm = np.cross(b - a, c - a)
            if np.dot(nrm, cen - a) > 0:
                nrm = -nrm
            assert np.all((pts - a) @ nrm <= 1e-9 * scale * np.linalg.norm(nrm) * scale)


def test_round6_matches_printf(oracle):
    """The %g rounding Qhull's input went through (LQRO:871-873)."""
    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.normal(size=2000) * 10.0 ** rng.integers(-6, 8, 2000),
                           [0.0, -0.0, 1e-5, 123456.5, 999999.5, 1e21, -2.5e-7]])
    for v in vals:
        assert oracle.round6(v) == float("%g" % v), v


def test_hull_cases_match_scipy_qhull(oracle):
    """The same inside-hull point sets against scipy's bundled Qhull
    (qhull_r 2019.1, which reproduces the reference's Qhull fixture above
    facet-for-facet): identical facet sets as canonical sorted triples."""
    spatial = pytest.importorskip("scipy.spatial")
    P = _load("pairs.npz")
    for h in range(int(P["n_hull"])):
        pts = np.vectorize(oracle.round6)(P[f"hull{h}_pts"])
        ours = sorted(tuple(sorted(int(v) for v in t)) for t in oracle.hull(pts))
        ref = sorted(tuple(sorted(int(v) for v in s)) for s in spatial.ConvexHull(pts).simplices)
        assert ours == ref, h


def test_pseudo_inverse_matches_reference(oracle):
    """pseudoInverse over jacobi2 (MAT:450-477, 887-1037), the kernel of l in
    controlMatrices (LQRO:552), against the reference build
    (tests/golden/pinv.npz: full rank, rank 4, symmetric, near-singular and
    the closed loop of the reference's own model), bit for bit."""
    d = _load("pinv.npz")
    for q, ref in zip(d["inputs"], d["outputs"]):
        got = oracle.pinv(q)
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))


def test_feedforward_l_matches_reference(oracle):
    """l of controlMatrices (LQRO:552-557) for the reference's model equals the
    reference's (tests/golden/dyn.npz, ref_gain_l), sign of zero included."""
    d = _load("dyn.npz")
    got = oracle.synthesize()["l"]
    assert np.array_equal(got.view(np.uint64), d["l"].view(np.uint64))
