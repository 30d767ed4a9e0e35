"""The oracle's restatement of Qhull's build (oracle/lqro_qhull.c) and the
reference's own hull rule over it (orc_hull_branch_ref, LQRObstacles.cpp:
867-969) — CPU.

qconvex.exe is never run; its stand-in is scipy's bundled Qhull 2019.1
called exactly like qconvex (tests/golden/qhull_lib.py), which
reproduces the reference's own fixture (tests/golden/qhull).  Pinned here:
  * orc_qhull against live Qhull: facet order, every facet's Fv vertex list,
    every plane bit for bit — on the reference's fixture, random clouds and
    path hulls;
  * the same against tests/golden/qhull_order.npz's Qhull output (no live
    Qhull needed);
  * the oracle's step with the reference's rule (planes read back as
    printed) against the golden reference loop, bit for bit: every inside
    pair's facet, distance and carried normal, every row's newV."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN

QO = os.path.join(GOLDEN, "qhull_order.npz")


def _live():
    sys.path.insert(0, GOLDEN)
    try:
        import qhull_lib
        qhull_lib._lib()
        return qhull_lib
    except Exception as e:   # scipy's Qhull internals not loadable here
        pytest.skip(f"live Qhull unavailable: {e}")


def _same_as_qhull(oracle, q, pts):
    st, fv, pl, _ = oracle.qhull(pts)
    assert st == 0
    planes, qfv, _, _ = q.qconvex(pts)
    assert [list(f) for f in qfv] == fv.tolist()
    from scipy.spatial import ConvexHull
    eq = ConvexHull(pts).equations          # the same build's unprinted planes
    assert np.array_equal(eq, pl)
    assert (np.abs(planes - pl) <= 1e-15 * np.maximum(1.0, np.abs(pl))).all()   # as printed (%.16g)


def test_oracle_qhull_on_reference_fixture(oracle):
    q = _live()
    _same_as_qhull(oracle, q, q.read_pointlist(os.path.join(GOLDEN, "qhull", "pointList.txt")))


def test_oracle_qhull_random_clouds(oracle):
    q = _live()
    rng = np.random.default_rng(3)
    for t in range(12):
        n = int(rng.integers(8, 400))
        pts = np.round(rng.normal(size=(n, 3)) * 10 ** rng.uniform(-1, 2), int(rng.integers(2, 6)))
        _same_as_qhull(oracle, q, pts)


def test_oracle_qhull_golden_hulls(oracle):
    """The six dense-swarm hulls stored with Qhull's output: no live Qhull."""
    d = np.load(QO)
    for k in range(6):
        st, fv, pl, _ = oracle.qhull(d[f"inject{k}_rounded"])
        assert st == 0
        assert np.array_equal(fv, d[f"inject{k}_fv"])
        g = d[f"inject{k}_planes"]
        assert (np.abs(pl[:, :4] - g) <= 1e-15 * np.maximum(1.0, np.abs(g))).all()


@pytest.mark.parametrize("case", ["dense", "c2"])
def test_oracle_reference_rule_step(oracle, lqro_mod, gains, case):
    d = np.load(QO)
    N, H, box, seed = (32, 45, 3.0, 11) if case == "dense" else (64, 50, None, None)
    x, vg = lqro_mod.synthetic_swarm(N, box=box, seed=seed) if box else lqro_mod.synthetic_swarm(N)
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    oracle.set_hull_rule(1, round16=True)
    oracle.carry_normal(np.zeros(3))
    try:
        v, r = oracle.step(T, NCF, oracle.sphere(100), x, vg, threads=4)
    finally:
        oracle.set_hull_rule(0)
    g = d[f"{case}_pairs"]
    ins = r[(r["flags"] & 2) != 0]
    assert np.array_equal(ins["i"], g["i"]) and np.array_equal(ins["j"], g["j"])
    assert np.array_equal(ins["facet"], g["fv"])
    assert np.array_equal(ins["dist"].view(np.uint64), g["dist"].view(np.uint64))
    assert np.array_equal(ins["normal"].view(np.uint64), g["normal"].view(np.uint64))
    assert np.array_equal((ins["flags"] & 0x40) != 0, g["stale"] != 0)
    assert np.array_equal(v.view(np.uint64), d[f"{case}_newv"].view(np.uint64))
    assert np.array_equal(oracle.carry_normal(), d[f"{case}_carry"])


def test_k_qhull_caps_and_the_wide_insertion(oracle, lqro_mod, gains):
    """k_qhull's per-insertion caps (csrc/lqro_qhull3.hpp) against the widest
    insertion of the crowded 30 m swarm (scripts/qhull_caps.py over its 421
    inside-hull pairs, oracle build statistics): pair (1018, 516) has one
    insertion with 166 visible and 116 new facets.  Round 3's Q3_VISCAP of 128
    sent that build to k_qhull_big (70 ms of the 30 m step's 108 ms hull
    phase, profiles/r3h_crowded30_plain_trace.txt); Q3_VISCAP = 192 (the LDS
    facet slots cut to 2,240 to make room) keeps it in k_qhull: every cap
    holds."""
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "lqr-obstacles_amd", "csrc", "lqro_qhull3.hpp")).read()
    cap = {k: int(re.search(rf"#define Q3_{k} (\d+)", src).group(1)) for k in ("VISCAP", "NEWCAP", "HZCAP", "COPCAP")}
    x, _ = lqro_mod.synthetic_swarm(1024, box=30.0)
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], 100)
    _, _, pts = oracle.pair(T, NCF, oracle.sphere(100), x[1018], x[516], 1018, 516, want_points=True)
    oracle.qhull(pts)
    st = oracle.last_qhull_stats
    assert st["st_visible_max"] == 166 and st["st_new_max"] == 116, st
    assert st["st_visible_max"] <= cap["VISCAP"] and st["st_new_max"] <= cap["NEWCAP"]
    assert st["st_horizon_max"] <= cap["HZCAP"] and st["st_cop_max"] <= cap["COPCAP"]


def test_oracle_flags_merged_winners(oracle):
    """tests/golden/qhull_merge.npz (live Qhull, make_golden_merge.py): inputs
    whose qconvex winner is a merged facet (coplanar cube faces, a flattened
    cap).  The oracle's merge-free restatement must flag them (Qhull's merge
    tests fired, and a facet within 1e-6 of the winning distance has another
    vertex on its plane: LQRO_REC_QHMERGE_WIN, reported as qstatus bit
    0x10000), and on the reference's fixture (no merge) it must not."""
    d = np.load(os.path.join(GOLDEN, "qhull_merge.npz"))
    oracle.set_hull_rule(1, round16=True)
    try:
        for c in ("cube_top", "cube_side", "capped"):
            e = d[f"{c}_expect"]
            off = d[f"{c}_fvoff"]
            assert e[1] == 1 and off[int(e[0]) + 1] - off[int(e[0])] > 3, c   # qconvex's winner is merged
            nf, dist, nrm, fac, qst = oracle.hull_branch_ref(d[f"{c}_pts"], d[f"{c}_vrel"])
            assert nf > 0 and (qst & 0x7f) and (qst & 0x10000), (c, hex(qst))
        from test_oracle_golden import _qhull_fixture
        pts, _, _ = _qhull_fixture()
        pts = np.ascontiguousarray(pts, np.float64)
        nf, dist, nrm, fac, qst = oracle.hull_branch_ref(pts, pts.mean(0))
        assert nf == 62 and qst == 0
    finally:
        oracle.set_hull_rule(0)
