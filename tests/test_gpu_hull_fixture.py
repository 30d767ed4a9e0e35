"""The GPU hulls on the reference's own Qhull fixture (tests/golden/qhull:
pointList.txt, the qconvex input LQRObstacles.cpp:869-880 writes, with
facetVertices.txt / Planes.txt, qconvex's output), through the test hook
lqro_debug_hull_points (not in lqro.h):

- k_hull (the full in-kernel quickhull) has exactly the fixture's 62 facets;
- k_hull and k_lhull (the local hull) select the oracle's
  facet and distance (orc_hull_branch, the rule of LQRO:925-967 as restated,
  §5.1) for relative velocities inside the hull, bit for bit."""
import ctypes as C

import numpy as np
import pytest

from test_oracle_golden import _qhull_fixture

pytestmark = pytest.mark.gpu


def _vrels(pts):
    cen = pts.mean(0)
    out = [cen]
    for k in (0, 100, 517, 1000):
        out.append(cen + 0.9 * (pts[k] - cen))
    return out


def test_gpu_hulls_on_reference_qhull_fixture(lqro_mod, oracle, gains):
    pts, planes, fv = _qhull_fixture()
    pts = np.ascontiguousarray(pts, np.float64)
    ref = sorted(tuple(sorted(f[1:])) for f in fv)
    L = lqro_mod.lib()
    L.lqro_debug_hull_points.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p,
                                         C.c_int32, C.POINTER(C.c_int32), C.POINTER(lqro_mod.PairRecord)]
    ctx = lqro_mod.Context(lqro_mod.config(2, 100, 100))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    try:
        for v in _vrels(pts):
            v = np.ascontiguousarray(v, np.float64)
            _, d_ref, _, fac = oracle.hull_branch(pts, v)
            got = {}
            for local in (0, 1):
                facets = np.zeros((4096, 3), np.int32)
                nf = C.c_int32(0)
                rec = lqro_mod.PairRecord()
                rc = L.lqro_debug_hull_points(ctx._h, pts.ctypes.data, pts.shape[0], v.ctypes.data, local,
                                              facets.ctypes.data, 4096, C.byref(nf), C.byref(rec))
                assert rc == 0
                if local == 0:
                    assert nf.value == len(ref)
                    assert sorted(tuple(sorted(t)) for t in facets[: nf.value].tolist()) == ref
                else:
                    assert nf.value == 0, "the local hull handed the fixture over"
                assert rec.flags & lqro_mod.REC_HULL
                got[local] = (sorted(rec.facet), rec.dist)
            assert got[0] == got[1] == (sorted(fac.tolist()), d_ref)
    finally:
        ctx.close()
