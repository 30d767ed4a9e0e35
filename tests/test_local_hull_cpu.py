"""The local-hull argument (k_lhull) on the CPU: the EPA-style
local hull around vrel (scripts/epa_spike.py: vrel strictly inside Q, window
facets and their 1-ring certified against every rounded point) selects the
full hull's canonical facet and distance, bit for bit, on every inside-hull
pair of the dense-swarm fixture (tests/golden/hull_rule.npz), with far fewer
vertices.  The GPU kernel is checked against the full hull in
tests/test_gpu_parity.py::test_local_hull_identical."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "lqr-obstacles_amd")]


def test_local_hull_matches_full_hull_dense():
    import epa_spike
    import lqro
    import pyoracle
    fx = np.load(os.path.join(ROOT, "tests", "golden", "hull_rule.npz"))
    g = pyoracle.synthesize()
    H = 45
    T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = pyoracle.sphere(100)
    x, _ = lqro.synthetic_swarm(32, box=3.0, seed=11)
    nloc, nfull = [], []
    for i, j in zip(fx["dense_i"], fx["dense_j"]):
        _, _, P = pyoracle.pair(T, NCF, S, x[i], x[j], int(i), int(j), want_points=True)
        R = np.vectorize(pyoracle.round6)(P)
        v = x[i, 3:6] - x[j, 3:6]
        _, d_full, _, fac = pyoracle.hull_branch(P, v)
        res = epa_spike.local(R, P, v)
        assert res is not None, (i, j)
        d_loc, t_best, nverts, _ = res
        assert d_loc == d_full and sorted(t_best) == sorted(fac.tolist()), (i, j)
        nloc.append(nverts)
        nfull.append(len({u for f in pyoracle.hull(R) for u in f}))
    assert len(nloc) == 92
    assert np.mean(nloc) < 0.5 * np.mean(nfull)
