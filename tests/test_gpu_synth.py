"""Batched gain synthesis on the GPU (lqro_synthesize_gains_batch, one agent
per lane): controlMatrices (LQRO:520-582) for heterogeneous agents (SURVEY §8f
next #2), bit-exact against the oracle's C restatement (itself pinned to the
reference's golden gains) and against the host path of the same source."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

KEYS = ("A", "B", "c", "L", "E", "l", "Lh", "Eh")


def perturbed_models(lqro_mod, n, seed=9, rel=0.01):
    """Agents whose mass, inertia, rotor latency, arm length and cost weights
    differ by up to +-1 % (C5's heterogeneous swarm)."""
    rng = np.random.default_rng(seed)
    ms = []
    for _ in range(n):
        m = lqro_mod.default_model()
        for f in ("mass", "inertia", "thrust_latency", "length", "qv", "qp", "r"):
            setattr(m, f, getattr(m, f) * (1.0 + rng.uniform(-rel, rel)))
        ms.append(m)
    return ms


def test_batch_synthesis_bit_exact(lqro_mod, oracle):
    models = perturbed_models(lqro_mod, 40)
    got = lqro_mod.synthesize_gains_batch(models)
    for k, m in enumerate(models):
        om = oracle.Model(*[getattr(m, f) for f, _ in m._fields_])
        ref = oracle.synthesize(om)
        host = lqro_mod.synthesize_gains(m)
        for key in KEYS:
            assert np.array_equal(got[key][k].view(np.uint64), ref[key].view(np.uint64)), (k, key)
            assert np.array_equal(host[key].view(np.uint64), ref[key].view(np.uint64)), (k, key)


def test_batch_default_model_is_golden(lqro_mod):
    ref = dict(np.load(os.path.join(GOLDEN, "gains.npz")))
    ref["l"] = np.load(os.path.join(GOLDEN, "dyn.npz"))["l"]      # ref_gain_l (LQRO:552-557)
    got = lqro_mod.synthesize_gains_batch([lqro_mod.default_model()] * 3)
    for key in KEYS:
        for k in range(3):
            assert np.array_equal(got[key][k].view(np.uint64), ref[key].view(np.uint64)), key


def test_heterogeneous_step_matches_oracle(lqro_mod, oracle):
    """Per-agent gains from the batch feed the per-agent tables (k_tables) and
    the step: rows bit-exact against the oracle with the same per-agent L, E."""
    N, H, NP = 24, 50, 100
    g = lqro_mod.synthesize_gains_batch(perturbed_models(lqro_mod, N, seed=4))
    x, vg = lqro_mod.synthetic_swarm(N)
    A, B = g["A"][0], g["B"][0]          # the shared linearisation the pair loop reads (LQRO:1265-1266)
    ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, flags=lqro_mod.LQRO_FLAG_RECORDS))
    ctx.set_gains(A, B, g["L"], g["E"], per_agent=True)
    newv = ctx.step(x, vg)
    recs = ctx.records()
    ctx.close()
    T = np.zeros((N, H, 9))
    NCF = np.zeros((N, H, 3, 16))
    for i in range(N):
        T[i], NCF[i] = oracle.tables(A, B, g["L"][i], g["E"][i], H)
    S = oracle.sphere(NP)
    rv, rr = oracle.step(T, NCF, S, x, vg, per_agent=True, threads=8)
    assert np.array_equal(recs["n_reach"], rr["n_reach"])
    assert np.array_equal(recs["reach_hash"], rr["reach_hash"])
    out = ((rr["flags"] & 1) != 0) & ((rr["flags"] & 2) == 0)
    assert np.array_equal(recs["dist"][out].view(np.uint64), rr["dist"][out].view(np.uint64))
    np.testing.assert_allclose(newv, rv, rtol=1e-5, atol=1e-6)
