"""BASELINE configs 4 and 5 on the HIP path, one GPU's shard each (the
8-GPU runs shard rows; every rank runs exactly this).

C4: 4096 quadrotors, H = 100, rows [0, 512) = one 8-way shard (2,096,640
    pairs), shared gains: every pair against the oracle (records bit-exact,
    hull pairs' arg-min facet and distance exact), newV exact on rows whose
    planes all match.
C5: 16384 agents with the 12-DoF reduced model (lqro_synthesize_gains_x,
    rotor-force states dropped), per-agent gains from ±1 %-perturbed models
    (lqro_synthesize_gains_batch_x), H = 200, rows [0, 2048) = one 8-way
    shard (33,552,384 pairs).  The whole shard runs on the GPU; the oracle
    checks newV on 32 rows spread over the shard and every record of 8 rows
    (131,064 pairs); full-size properties: no hull failure, finite newV, the
    same result from a second step.  No reference exists for X = 12 (SURVEY
    §7 hazard 7): the oracle's restatement of the reduced model pins the GPU
    synthesis bit for bit.
"""
import numpy as np
import pytest

from test_gpu_parity import _compare, _flags, _hull_pairs_equal, _oracle_step

pytestmark = pytest.mark.gpu

KEYS = ("A", "B", "c", "L", "E", "l", "Lh", "Eh")


def _oracle_model(oracle, m):
    return oracle.Model(*[getattr(m, f) for f, _ in m._fields_])


def _hull_exact(recs, rrecs):
    inside = (rrecs["flags"] & 2) != 0
    assert np.all(recs["flags"][inside] & 8), "hull failed"
    assert np.array_equal(recs["facet"][inside], rrecs["facet"][inside])
    assert np.array_equal(recs["dist"][inside].view(np.uint64), rrecs["dist"][inside].view(np.uint64))
    return inside


@pytest.mark.parametrize("rule", ["qhull", "canonical"])
def test_c4_shard(lqro_mod, oracle, gains, rule):
    """C4's first 8-way shard in both inside-hull rules (Qhull order, the
    default: k_qhull, the carried normal entering the shard 0 as for rank 0)."""
    N, H, NP, rows = 4096, 100, 100, (0, 512)
    x, vg = lqro_mod.synthetic_swarm(N)
    ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, row_begin=rows[0], row_end=rows[1],
                                           flags=_flags(lqro_mod, rule)))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    newv = ctx.step(x, vg)
    recs = ctx.records()
    st = ctx.stats()
    ctx.close()
    assert st["pairs"] == 512 * 4095 and st["hull_fail"] == 0
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    rv, rrecs = _oracle_step(oracle, rule, T, NCF, oracle.sphere(NP), x, vg, rows=rows, threads=16)
    _compare(recs, rrecs)
    inside = _hull_pairs_equal(lqro_mod, recs, rrecs, rule)
    assert inside.sum() > 0
    clean = np.ones(N, bool)
    clean[rrecs["i"][inside]] = False
    clean[:rows[0]] = clean[rows[1]:] = False
    assert np.array_equal(newv[clean], rv[clean])
    np.testing.assert_allclose(newv[rows[0]:rows[1]], rv[rows[0]:rows[1]], rtol=1e-5, atol=1e-6)


def test_reduced_model_synthesis_bit_exact(lqro_mod, oracle):
    """X = 12 gains: the GPU batch (one agent per lane) and the host path of
    the same source against the oracle's C restatement, ±1 % models."""
    models = lqro_mod.perturbed_models(48)
    got = lqro_mod.synthesize_gains_batch(models, x_dim=12)
    assert got["A"].shape == (48, 12, 12) and got["L"].shape == (48, 4, 12)
    for k, m in enumerate(models):
        ref = oracle.synthesize(_oracle_model(oracle, m), x_dim=12)
        host = lqro_mod.synthesize_gains(m, x_dim=12)
        for key in KEYS:
            assert np.array_equal(got[key][k].view(np.uint64), ref[key].view(np.uint64)), (k, key)
            assert np.array_equal(host[key].view(np.uint64), ref[key].view(np.uint64)), (k, key)
    # the reduced model is the 16-state one without the rotor lag: position,
    # velocity and attitude blocks of the closed loop stay stable
    g16 = oracle.synthesize(x_dim=16)
    g12 = oracle.synthesize(x_dim=12)
    for g, X in ((g16, 16), (g12, 12)):
        acl = g["A"] + g["B"] @ g["L"]
        assert np.abs(np.linalg.eigvals(acl)).max() < 1.0 + 1e-6, X


@pytest.fixture(scope="module")
def c5(lqro_mod):
    N, H, NP, X = 16384, 200, 100, 12
    models = lqro_mod.perturbed_models(N)
    g = lqro_mod.synthesize_gains_batch(models, x_dim=X)
    A, B = lqro_mod.synthesize_gains(x_dim=X)["A"], lqro_mod.synthesize_gains(x_dim=X)["B"]
    x, vg = lqro_mod.synthetic_swarm(N, x_dim=X)
    return dict(N=N, H=H, NP=NP, X=X, A=A, B=B, L=g["L"], E=g["E"], x=x, vg=vg)


def _c5_ctx(lqro_mod, c, rows, records=False):
    ctx = lqro_mod.Context(lqro_mod.config(c["N"], c["H"], c["NP"], x_dim=c["X"], row_begin=rows[0],
                                           row_end=rows[1],
                                           flags=lqro_mod.LQRO_FLAG_RECORDS if records else 0))
    ctx.set_gains(c["A"], c["B"], c["L"], c["E"], per_agent=True)
    return ctx


def test_c5_shard(lqro_mod, oracle, c5):
    c = c5
    rows = (0, 2048)
    ctx = _c5_ctx(lqro_mod, c, rows)
    newv = ctx.step(c["x"], c["vg"])
    st = ctx.stats()
    newv2 = ctx.step(c["x"], c["vg"])
    tm = ctx.timings()
    ctx.close()
    print(f"C5 shard: {st}, {tm}")
    assert st["pairs"] == 2048 * 16383
    assert st["hull_fail"] == 0 and st["inside"] > 0
    own = newv[rows[0]:rows[1]]
    assert np.isfinite(own).all()
    assert np.array_equal(newv2, newv)
    S = oracle.sphere(c["NP"])
    for r in range(7, 2048, 64):       # 32 rows over the shard, row r's own tables
        T, NCF = oracle.tables(c["A"], c["B"], c["L"][r], c["E"][r], c["H"], X=c["X"])
        rv, _ = oracle.step(T, NCF, S, c["x"], c["vg"], rows=(r, r + 1), threads=16, records=False)
        np.testing.assert_allclose(newv[r], rv[r], rtol=1e-5, atol=1e-6, err_msg=f"row {r}")


def test_c5_rows_records(lqro_mod, oracle, c5):
    c = c5
    rows = (1024, 1032)
    ctx = _c5_ctx(lqro_mod, c, rows, records=True)
    newv = ctx.step(c["x"], c["vg"])
    recs = ctx.records()
    ctx.close()
    S = oracle.sphere(c["NP"])
    T = np.zeros((c["N"], c["H"], 9))
    NCF = np.zeros((c["N"], c["H"], 3, c["X"]))
    for r in range(*rows):
        T[r], NCF[r] = oracle.tables(c["A"], c["B"], c["L"][r], c["E"][r], c["H"], X=c["X"])
    rv, rrecs = oracle.step(T, NCF, S, c["x"], c["vg"], rows=rows, per_agent=True, threads=16)
    _compare(recs, rrecs)
    _hull_exact(recs, rrecs)
    np.testing.assert_allclose(newv[rows[0]:rows[1]], rv[rows[0]:rows[1]], rtol=1e-5, atol=1e-6)


def test_c5_qhull_order_largest_hulls(lqro_mod, oracle, c5):
    """Qhull order (the default rule) on C5: a shard with hulls of ~19,000
    points whose single insertions see more than 256 visible and new facets
    (k_qhull_big, QH_VISCAP / QH_NEWCAP) builds every hull; three such rows
    against the oracle's restatement of Qhull's build, bit for bit."""
    c = c5
    ctx = lqro_mod.Context(lqro_mod.config(c["N"], c["H"], c["NP"], x_dim=c["X"], row_begin=2048, row_end=4096,
                                           flags=lqro_mod.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(c["A"], c["B"], c["L"], c["E"], per_agent=True)
    try:
        ctx.step(c["x"], c["vg"])
    except lqro_mod.QhullMergeSuspect as e:   # reported loudly, never silent (LQRO_E_QHMERGE)
        assert len(e.pairs) > 0
    st = ctx.stats()
    ctx.close()
    assert st["hull_fail"] == 0 and st["inside"] > 500, st
    assert st["qhull_merge_win"] <= 2, st   # (the whole C5 swarm, sampled: 1 of 4,867, profiles/r6_qhmerge_c5_scan.txt)
    S = oracle.sphere(c["NP"])
    oracle.set_hull_rule(1, round16=True)
    try:
        for r in (3014, 3155, 5156):
            ctx = lqro_mod.Context(lqro_mod.config(c["N"], c["H"], c["NP"], x_dim=c["X"], row_begin=r, row_end=r + 1,
                                                   flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER))
            ctx.set_gains(c["A"], c["B"], c["L"], c["E"], per_agent=True)
            try:
                newv = ctx.step(c["x"], c["vg"])
            except lqro_mod.QhullMergeSuspect as e:   # (flagged alike by the oracle: compared below)
                newv = e.newv
            recs = ctx.records()
            ctx.close()
            T = np.zeros((c["N"], c["H"], 9))
            NCF = np.zeros((c["N"], c["H"], 3, c["X"]))
            T[r], NCF[r] = oracle.tables(c["A"], c["B"], c["L"][r], c["E"][r], c["H"], X=c["X"])
            oracle.carry_normal(np.zeros(3))
            rv, rrecs = oracle.step(T, NCF, S, c["x"], c["vg"], rows=(r, r + 1), per_agent=True, threads=16)
            ins = (rrecs["flags"] & lqro_mod.REC_INSIDE) != 0
            assert ins.any() and not (recs["flags"][ins] & lqro_mod.REC_HULLFAIL).any(), r
            for f in ("facet", "dist", "normal", "plane_point", "plane_normal"):
                assert np.array_equal(recs[f][ins], rrecs[f][ins]), (r, f)
            assert np.array_equal(newv[r].view(np.uint64), rv[r].view(np.uint64)), r
    finally:
        oracle.set_hull_rule(0)
