"""The reference-faithful oracle mode (orc_step_faithful_mt, the CPU baseline
bench.py times): the reference's per-pair cost structure — findFG recursion
per pair (LQRO:1401-1406) and GJK run twice for an outside pair
(LQRO:1410/1414) — with results bit-identical to the hoisted oracle step,
for shared and per-agent gains and X = 12."""
import numpy as np
import pytest


@pytest.mark.parametrize("X,per_agent", [(16, False), (16, True), (12, True)])
def test_faithful_equals_hoisted(oracle, lqro_mod, X, per_agent):
    N, H, NP = 14, 40, 50
    x, vg = lqro_mod.synthetic_swarm(N, box=4.0, seed=5, x_dim=X)
    S = oracle.sphere(NP)
    if per_agent:
        gs = [oracle.synthesize(oracle.Model(*[getattr(m, f) for f, _ in m._fields_]), x_dim=X)
              for m in lqro_mod.perturbed_models(N, seed=3)]
        A, B = gs[0]["A"], gs[0]["B"]
        L = np.stack([g["L"] for g in gs])
        E = np.stack([g["E"] for g in gs])
        T = np.zeros((N, H, 9))
        NCF = np.zeros((N, H, 3, X))
        for i in range(N):
            T[i], NCF[i] = oracle.tables(A, B, L[i], E[i], H, X=X)
    else:
        g = oracle.synthesize(x_dim=X)
        A, B, L, E = g["A"], g["B"], g["L"], g["E"]
        T, NCF = oracle.tables(A, B, L, E, H, X=X)
    v0, r0 = oracle.step(T, NCF, S, x, vg, per_agent=per_agent)
    v1, r1 = oracle.step_faithful(A, B, L, E, S, x, vg, H, per_agent=per_agent, threads=3)
    assert (r0["flags"] & 1).sum() > 0
    assert np.array_equal(v0.view(np.uint64), v1.view(np.uint64))
    for f in r0.dtype.names:
        assert np.array_equal(r0[f], r1[f]), f
