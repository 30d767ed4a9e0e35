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
