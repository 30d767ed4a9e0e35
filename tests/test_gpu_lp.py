"""GPU new-velocity LP (lqro_calculate_new_v, one wavefront per agent) vs the
oracle's sequential fp32 restatement of calculateNewV: bit-exact."""
import numpy as np
import pytest

from lp_cases import random_cases

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,max_planes", [(1, 60), (2, 200), (3, 1100)])
def test_lp_bit_exact(lqro_mod, oracle, seed, max_planes):
    cases, goals = random_cases(300 if max_planes < 500 else 60, seed=seed, max_planes=max_planes)
    got = lqro_mod.calculate_new_v(cases, goals)
    ref = np.array([oracle.newv(c, g) for c, g in zip(cases, goals)])
    bad = np.where(~np.all(got == ref, axis=1))[0]
    assert bad.size == 0, (bad[:10], got[bad[:3]], ref[bad[:3]])


def test_lp_c3_hardest_rows(lqro_mod):
    """The C3 swarm's slowest linearProgram4 rows (tests/golden/lp_rows.npz,
    1,023 planes each, made by make_golden_lp_rows.py from the oracle step
    that qhull_order.npz pins): bit-exact new velocities."""
    import os
    from conftest import GOLDEN
    d = np.load(os.path.join(GOLDEN, "lp_rows.npz"))
    got = lqro_mod.calculate_new_v(list(d["planes"]), d["vgoal"], vmax_lp=float(d["vmax_lp"]))
    assert np.array_equal(got.view(np.uint64), d["newv"].view(np.uint64))
