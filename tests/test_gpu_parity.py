"""GPU parity: liblqro.so's HIP path vs the CPU oracle on identical inputs.

Bar: integer outputs (n_reach, reachable-set hash, inside
flag, GJK simplex, hull arg-min facet) bit-exact; fp64 GJK outputs and the
fp32 half-planes bit-exact on the non-hull branch (same operation order);
newV (fp32 LP) bit-exact when every plane matches.

Tests marked with the `rule` parameter run both inside-hull rules: "qhull",
the default (LQRO_FLAG_QHULL_ORDER: Qhull's build order, first Fv vertex,
the loop-carried normal, k_qhull) against the oracle in set_hull_rule(1),
and "canonical" (the opt-in local-hull rule) against the oracle's default.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RULES = ("qhull", "canonical")


def _flags(lqro_mod, rule):
    return lqro_mod.LQRO_FLAG_RECORDS | (lqro_mod.LQRO_FLAG_QHULL_ORDER if rule == "qhull" else 0)


def _oracle_step(oracle, rule, *a, **kw):
    """oracle.step under the hull rule (Qhull order: the carried normal
    entering the step is 0, as a fresh context's)."""
    if rule == "qhull":
        oracle.set_hull_rule(1, round16=True)
        oracle.carry_normal(np.zeros(3))
    try:
        return oracle.step(*a, **kw)
    finally:
        oracle.set_hull_rule(0)


def _run(lqro_mod, oracle, gains, x, vg, H, NP, rows=None, rule="canonical"):
    N = x.shape[0]
    kw = dict(flags=_flags(lqro_mod, rule))
    if rows is not None:
        kw.update(row_begin=rows[0], row_end=rows[1])
    ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, **kw))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    newv = ctx.step(x, vg)
    recs = ctx.records()
    st = ctx.stats()
    ctx.close()
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    S = oracle.sphere(NP)
    rv, rrecs = _oracle_step(oracle, rule, T, NCF, S, x, vg, rows=rows, threads=8)
    return newv, recs, st, rv, rrecs


def _hull_pairs_equal(lqro_mod, recs, rrecs, rule):
    """Every inside-hull pair: a plane was built, the arg-min facet (Fv order
    in Qhull order), the distance and the normal bit for bit; in Qhull order
    also the stale-normal flag and the facet count."""
    inside = (rrecs["flags"] & 2) != 0
    assert np.all(recs["flags"][inside] & 8), "hull failed"
    assert np.array_equal(recs["facet"][inside], rrecs["facet"][inside])
    assert np.array_equal(recs["dist"][inside].view(np.uint64), rrecs["dist"][inside].view(np.uint64))
    assert np.array_equal(recs["normal"][inside].view(np.uint64), rrecs["normal"][inside].view(np.uint64))
    if rule == "qhull":
        st = lqro_mod.REC_STALE
        assert np.array_equal(recs["flags"][inside] & st, rrecs["flags"][inside] & st)
        assert np.array_equal(recs["n_facets"][inside], rrecs["n_facets"][inside])
        assert np.array_equal(recs["plane_point"][inside].view(np.uint32), rrecs["plane_point"][inside].view(np.uint32))
    return inside


def _compare(recs, rrecs):
    assert np.array_equal(recs["i"], rrecs["i"]) and np.array_equal(recs["j"], rrecs["j"])
    assert np.array_equal(recs["n_reach"], rrecs["n_reach"])
    assert np.array_equal(recs["reach_hash"], rrecs["reach_hash"])
    assert np.array_equal(recs["flags"] & 3, rrecs["flags"] & 3)
    out = (rrecs["flags"] & 1) & ~((rrecs["flags"] >> 1) & 1)
    o = out.astype(bool)
    for f in ("gjk_iters", "simplex_n", "simplex", "dist", "normal", "wpt_vrel", "wpt_hull",
              "plane_point", "plane_normal"):
        a, b = recs[f][o], rrecs[f][o]
        if a.dtype.kind == "f":
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), f
        else:
            assert np.array_equal(a, b), f
    return o


@pytest.mark.parametrize("rule", RULES)
@pytest.mark.parametrize("N,H,NP", [(4, 50, 100), (24, 50, 100), (16, 100, 100), (10, 200, 50)])
def test_step_bit_exact(lqro_mod, oracle, gains, N, H, NP, rule):
    x, vg = lqro_mod.synthetic_swarm(N)
    newv, recs, st, rv, rrecs = _run(lqro_mod, oracle, gains, x, vg, H, NP, rule=rule)
    o = _compare(recs, rrecs)
    _hull_pairs_equal(lqro_mod, recs, rrecs, rule)
    inside = (rrecs["flags"] & 2) != 0
    rows_clean = np.ones(N, bool)
    for r in rrecs[inside]:
        rows_clean[r["i"]] = False
    assert np.array_equal(newv[rows_clean], rv[rows_clean])


@pytest.mark.parametrize("rule", RULES)
def test_c2_swarm(lqro_mod, oracle, gains, rule):
    """C2: 64 quadrotors, horizon 50 (4032 pairs)."""
    x, vg = lqro_mod.synthetic_swarm(64)
    newv, recs, st, rv, rrecs = _run(lqro_mod, oracle, gains, x, vg, 50, 100, rule=rule)
    _hull_pairs_equal(lqro_mod, recs, rrecs, rule)
    _compare(recs, rrecs)
    assert st["pairs"] == 64 * 63
    inside = (rrecs["flags"] & 2) != 0
    # hull branch: arg-min facet exact, distance/normal to the oracle's hull
    for r, q in zip(recs[inside], rrecs[inside]):
        assert r["flags"] & 8, "hull failed"
        assert np.array_equal(r["facet"], q["facet"])
        assert r["dist"] == q["dist"]
        assert np.array_equal(r["normal"], q["normal"])
    assert np.allclose(newv, rv, rtol=1e-5, atol=1e-7)


def test_row_shards_partition(lqro_mod, oracle, gains):
    """Rows [8, 20) of a 24-agent step equal the same rows of the full step."""
    x, vg = lqro_mod.synthetic_swarm(24, seed=7)
    newv, recs, st, rv, rrecs = _run(lqro_mod, oracle, gains, x, vg, 30, 50, rows=(8, 20))
    _compare(recs, rrecs)
    assert np.array_equal(newv[8:20], rv[8:20])


@pytest.mark.parametrize("world", [2, 3])
def test_cyclic_row_shards(lqro_mod, gains, world):
    """Cyclic sharding (row_stride = world): each rank's records and newV
    rows equal the same rows of the unsharded GPU step, on a dense swarm so
    the hull queue, the hot schedule and the LP all see strided rows."""
    N, H, NP = 30, 45, 100
    x, vg = lqro_mod.synthetic_swarm(N, box=3.0, seed=11)

    def run(**kw):
        ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, flags=lqro_mod.LQRO_FLAG_RECORDS, **kw))
        ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
        nv = ctx.step(x, vg)
        out = nv, ctx.records(), ctx.stats(), ctx.row_ids
        ctx.close()
        return out

    full_v, full_r, full_st, _ = run()
    assert full_st["inside"] > 0
    seen = 0
    for r in range(world):
        nv, rec, st, ids = run(**lqro_mod.shard_rows(N, r, world, "cyclic"))
        assert np.array_equal(ids, np.arange(r, N, world))
        sel = np.isin(full_r["i"], ids)
        ref = full_r[sel]
        _compare(rec, ref)
        inside = (ref["flags"] & 2) != 0
        assert np.all(rec["flags"][inside] & 8)
        assert np.array_equal(rec["facet"][inside], ref["facet"][inside])
        assert np.array_equal(rec["dist"].view(np.uint64), ref["dist"].view(np.uint64))
        assert np.array_equal(nv[ids], full_v[ids])
        others = np.setdiff1d(np.arange(N), ids)
        assert not nv[others].any()
        seen += st["pairs"]
    assert seen == N * (N - 1)


@pytest.mark.parametrize("rule", RULES)
def test_dense_swarm_inside_hull(lqro_mod, oracle, gains, rule):
    """A tight swarm (collision courses) exercises the in-kernel hull."""
    x, vg = lqro_mod.synthetic_swarm(32, box=3.0, seed=11)
    newv, recs, st, rv, rrecs = _run(lqro_mod, oracle, gains, x, vg, 45, 100, rule=rule)
    _compare(recs, rrecs)
    inside = _hull_pairs_equal(lqro_mod, recs, rrecs, rule)
    assert inside.sum() > 0
    if rule == "qhull":   # every plane equals the oracle's: so does every row's LP
        assert np.array_equal(newv.view(np.uint64), rv.view(np.uint64))


@pytest.mark.parametrize("rule", RULES)
@pytest.mark.parametrize("H", [200, 240, 256])
def test_large_horizon_hull(lqro_mod, oracle, gains, H, rule):
    """Canonical rule: H*NP = 20000 (C5's hull size) runs in k_hull, the LDS
    topology with its widened outside-set extents; H*NP > 21845 runs every
    hull job in k_hull_big (topology in global memory).  Qhull order: k_qhull
    for every size (k_qhull_big beyond its per-insertion caps).  Facets,
    distances and normals must match the oracle either way."""
    x, vg = lqro_mod.synthetic_swarm(8, box=2.5, seed=5)
    newv, recs, st, rv, rrecs = _run(lqro_mod, oracle, gains, x, vg, H, 100, rule=rule)
    _compare(recs, rrecs)
    inside = _hull_pairs_equal(lqro_mod, recs, rrecs, rule)
    assert inside.any()


def test_c3_full_step(lqro_mod, oracle, gains):
    """C3, the bench workload (1024 agents, H = 100, NP = 100: 1,047,552
    pairs), against the oracle: every non-hull pair bit-exact (this size
    reaches GJK's backup procedure), every hull pair's arg-min facet and
    distance exact, and newV bit-exact on rows without hull pairs."""
    N, H, NP = 1024, 100, 100
    x, vg = lqro_mod.synthetic_swarm(N)
    ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, flags=lqro_mod.LQRO_FLAG_RECORDS))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    newv = ctx.step(x, vg)
    recs = ctx.records()
    st = ctx.stats()
    ctx.close()
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    S = oracle.sphere(NP)
    rv, rrecs = oracle.step(T, NCF, S, x, vg, threads=16)
    _compare(recs, rrecs)
    assert st["gjk_backups"] == int(((rrecs["flags"] & 4) != 0).sum())
    inside = (rrecs["flags"] & 2) != 0
    assert inside.sum() > 100
    assert np.all(recs["flags"][inside] & 8), "hull failed"
    assert np.array_equal(recs["facet"][inside], rrecs["facet"][inside])
    assert np.array_equal(recs["dist"][inside], rrecs["dist"][inside])
    rows_clean = np.ones(N, bool)
    rows_clean[rrecs["i"][inside]] = False
    assert np.array_equal(newv[rows_clean], rv[rows_clean])
    np.testing.assert_allclose(newv, rv, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("kind", ["shared", "per_agent", "per_agent_x12_h200"])
def test_overlap_schedule_identical(lqro_mod, gains, monkeypatch, kind):
    """The step's schedule (k_prio hot list, side-stream hulls, side width,
    hot radius) changes only the order of work: every record and every new
    velocity is bit-identical across schedules and repeated steps — with
    shared gains (hot pairs on staged tables), per-agent gains (hot pairs read
    their row's tables from global memory) and C5's shape (X = 12, H = 200:
    k_side sweeps rows with the waves whose LDS regions fit)."""
    N, H, NP, X = 512, 100, 100, 16   # 261,632 pairs: the overlap path is taken
    per_agent = kind != "shared"
    if kind == "per_agent_x12_h200":
        H, X = 200, 12
    x, vg = lqro_mod.synthetic_swarm(N, seed=3, x_dim=X)
    if per_agent:
        g = lqro_mod.synthesize_gains_batch(lqro_mod.perturbed_models(N, seed=17), x_dim=X)
        gains = dict(A=g["A"][0], B=g["B"][0], L=g["L"], E=g["E"])
    outs = []
    for env in ({"LQRO_HOT": "0"}, {"LQRO_HOT": "1"}, {"LQRO_HOT": "1", "LQRO_SIDE_HULL_CUS": "32"},
                {"LQRO_HOT": "1", "LQRO_HOT_R": "0.5"}):
        for k in ("LQRO_HOT", "LQRO_SIDE_HULL_CUS", "LQRO_HOT_R"):
            monkeypatch.delenv(k, raising=False)
        monkeypatch.setenv("LQRO_LOCAL_HULL", "0")   # the overlap runs with the full hull only
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, x_dim=X, flags=lqro_mod.LQRO_FLAG_RECORDS))
        ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"], per_agent=per_agent)
        v1 = ctx.step(x, vg)
        r1 = ctx.records()
        v2 = ctx.step(x, vg)
        ctx.close()
        assert np.array_equal(v1, v2)
        outs.append((v1, r1))
    v0, r0 = outs[0]
    assert ((r0["flags"] & 2) != 0).sum() > 0
    for v, r in outs[1:]:
        assert np.array_equal(v, v0)
        for f in ("n_reach", "reach_hash", "flags", "facet", "dist", "normal", "plane_point", "plane_normal"):
            assert np.array_equal(r[f], r0[f]), f


def test_adaptive_schedule_identical(lqro_mod, gains, monkeypatch):
    """The schedule adapts to the inside-hull count of an earlier step: a
    crowded swarm (1024 agents in a 22 m box, ~1,100 inside-hull pairs) takes
    the plain schedule from its third step on (a step is scheduled by the
    count of the step two before it), a moderately dense one (30 m, ~420) a
    widened side stream.  Records and new velocities of those steps
    equal the plain schedule's and the forced overlap's bit for bit."""
    N, H, NP = 1024, 100, 100
    for box in (22.0, 30.0):
        x, vg = lqro_mod.synthetic_swarm(N, box=box, seed=7)
        outs = []
        for env in ({"LQRO_HOT": "0"}, {}, {"LQRO_HOT_MAX_INSIDE": "1000000"}):
            for k in ("LQRO_HOT", "LQRO_SIDE_HULL_CUS", "LQRO_HOT_R", "LQRO_HOT_MAX_INSIDE"):
                monkeypatch.delenv(k, raising=False)
            monkeypatch.setenv("LQRO_LOCAL_HULL", "0")
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, flags=lqro_mod.LQRO_FLAG_RECORDS))
            ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
            ctx.step(x, vg)                  # the count steps 3 and 4 are scheduled by
            ctx.step(x, vg)
            v = ctx.step(x, vg)
            r = ctx.records()
            v3 = ctx.step(x, vg)
            st = ctx.stats()
            ctx.close()
            assert np.array_equal(v, v3)
            assert st["hull_fail"] == 0
            outs.append((v, r, st["inside"]))
        v0, r0, n_in = outs[0]
        assert n_in > (300 if box == 30.0 else 800)
        for v, r, _ in outs[1:]:
            assert np.array_equal(v, v0)
            for f in ("n_reach", "reach_hash", "flags", "facet", "dist", "normal", "plane_point", "plane_normal"):
                assert np.array_equal(r[f], r0[f]), f


@pytest.mark.parametrize("rule", RULES)
@pytest.mark.parametrize("case", ["two_agents", "far_apart", "max_horizon"])
def test_edge_cases(lqro_mod, oracle, gains, case, rule):
    """Edge sizes: a single pair each way; a swarm so sparse that no pair
    emits a plane (every LP sees zero planes); the largest horizon the kernels
    take (H = 256 slices, 4 per lane) with NP = 50."""
    if case == "two_agents":
        x, vg = lqro_mod.synthetic_swarm(2, box=1.5, seed=2)
        H, NP = 50, 100
    elif case == "far_apart":
        x, vg = lqro_mod.synthetic_swarm(6, box=4000.0, seed=3)
        H, NP = 30, 50
    else:
        x, vg = lqro_mod.synthetic_swarm(6, box=4.0, seed=4)
        H, NP = 256, 50
    newv, recs, st, rv, rrecs = _run(lqro_mod, oracle, gains, x, vg, H, NP, rule=rule)
    _compare(recs, rrecs)
    if case == "far_apart":
        assert st["planes"] == 0 and st["inside"] == 0
    _hull_pairs_equal(lqro_mod, recs, rrecs, rule)
    np.testing.assert_allclose(newv, rv, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("scenario", ["swap", "c2", "dense"])
def test_reference_driver_one_call(lqro_mod, gains, scenario):
    """lqro_step against the reference's whole pair loop over all rows in one
    call (tests/golden/driver.npz, LQRO:1391-1436 with its loop-carried
    state): every row the reference harness completes, bit for bit."""
    import os
    from conftest import GOLDEN
    d = np.load(os.path.join(GOLDEN, "driver.npz"))
    H = int(d[f"{scenario}_H"])
    x, vg = d[f"{scenario}_x"], d[f"{scenario}_vgoal"]
    ctx = lqro_mod.Context(lqro_mod.config(x.shape[0], H, 100))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    newv = ctx.step(x, vg)
    ctx.close()
    ok = d[f"{scenario}_ok"].astype(bool)
    assert np.array_equal(newv[ok].view(np.uint64), d[f"{scenario}_newv"][ok].view(np.uint64))


@pytest.mark.parametrize("case", ["dense", "c3", "crowded", "x12_h200"])
def test_local_hull_identical(lqro_mod, gains, monkeypatch, case):
    """k_lhull (the inside-hull branch from a local hull around vrel,
    lqro_lhull.hpp) against the full hull (LQRO_LOCAL_HULL=0): every record
    (facet, distance, normal, half-plane) and every new velocity bit for bit,
    on a dense swarm, the C3 bench swarm, a crowded C3-sized swarm (22 m box,
    ~1,100 inside-hull pairs) and C5's shape (X = 12, H = 200, per-agent
    gains); the local hull decides nearly every inside pair (the rest are
    handed to k_hull), in the overlapped schedule (k_pair hot -> k_lhull ->
    k_pair rows on the side stream) and, for crowded swarms, the plain one."""
    import ctypes as C
    N, H, NP, X, box, seed, per_agent = 1024, 100, 100, 16, None, None, False
    if case == "dense":
        N, H, box, seed = 32, 45, 3.0, 11
    elif case == "crowded":
        box, seed = 22.0, 7
    elif case == "x12_h200":
        N, H, X, box, seed, per_agent = 256, 200, 12, 12.0, 5, True
    kw = {} if box is None else dict(box=box, seed=seed)
    lqro_mod.lib().lqro_debug_local_hull.argtypes = [C.c_void_p, C.c_void_p]
    x, vg = lqro_mod.synthetic_swarm(N, x_dim=X, **kw)
    g = gains
    if per_agent:
        gb = lqro_mod.synthesize_gains_batch(lqro_mod.perturbed_models(N, seed=17), x_dim=X)
        g = dict(A=gb["A"][0], B=gb["B"][0], L=gb["L"], E=gb["E"])
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("LQRO_LOCAL_HULL", flag)
        ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, x_dim=X, flags=lqro_mod.LQRO_FLAG_RECORDS))
        ctx.set_gains(g["A"], g["B"], g["L"], g["E"], per_agent=per_agent)
        v = ctx.step(x, vg)
        r = ctx.records()
        if flag == "1":
            # a third step is scheduled by the first's inside-hull count
            # (side width, or the plain schedule for crowded swarms)
            assert np.array_equal(ctx.step(x, vg), v)
            assert np.array_equal(ctx.step(x, vg), v)
            r2 = ctx.records()
            for f in ("flags", "facet", "dist", "plane_point", "plane_normal"):
                assert np.array_equal(r2[f], r[f]), f
        st = ctx.stats()
        out = (C.c_longlong * 18)()
        assert lqro_mod.lib().lqro_debug_local_hull(ctx._h, out) == 0
        ctx.close()
        outs.append((v, r, st, tuple(out)))
    (v0, r0, st0, _), (v1, r1, st1, out) = outs
    done, handed, reasons = out[0], out[1], out[2:]
    inside = (r0["flags"] & 2) != 0
    assert inside.sum() > 0 and st0["hull_fail"] == 0 and st1["hull_fail"] == 0
    local = (r1["flags"] & lqro_mod.REC_LOCAL) != 0
    assert local.sum() == done and done + handed == inside.sum()
    print(f"{case}: {inside.sum()} inside pairs, local hull decided {done}, handed over {handed} "
          f"(reasons {dict((k + 20, c) for k, c in enumerate(reasons) if c)})")
    assert np.array_equal(r1["flags"] & ~lqro_mod.REC_LOCAL, r0["flags"])
    for f in ("n_reach", "reach_hash", "facet", "dist", "normal", "plane_point", "plane_normal"):
        a, b = r1[f][inside], r0[f][inside]
        if a.dtype.kind == "f":
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), f
        else:
            assert np.array_equal(a, b), f
    assert np.array_equal(v1.view(np.uint64), v0.view(np.uint64))
    assert done >= 0.8 * inside.sum()


@pytest.mark.parametrize("kind", ["per_agent", "per_agent_x12_h200"])
def test_qhull_order_per_agent_gains(lqro_mod, oracle, kind):
    """The default rule (Qhull order) with per-agent gains from +-1 %-perturbed
    models, X = 16 and config 5's X = 12 / H = 200, on a dense swarm against
    the oracle: every record of every pair bit for bit, newV too."""
    N, H, X = 24, 100, 16
    if kind == "per_agent_x12_h200":
        H, X = 200, 12
    x, vg = lqro_mod.synthetic_swarm(N, box=4.0, seed=9, x_dim=X)
    g = lqro_mod.synthesize_gains_batch(lqro_mod.perturbed_models(N, seed=17), x_dim=X)
    A, B, L, E = g["A"][0], g["B"][0], g["L"], g["E"]
    ctx = lqro_mod.Context(lqro_mod.config(N, H, 100, x_dim=X, flags=_flags(lqro_mod, "qhull")))
    ctx.set_gains(A, B, L, E, per_agent=True)
    newv = ctx.step(x, vg)
    recs = ctx.records()
    ctx.close()
    T = np.zeros((N, H, 9))
    NCF = np.zeros((N, H, 3, X))
    for i in range(N):
        T[i], NCF[i] = oracle.tables(A, B, L[i], E[i], H, X=X)
    rv, rrecs = _oracle_step(oracle, "qhull", T, NCF, oracle.sphere(100), x, vg, per_agent=True, threads=8)
    _compare(recs, rrecs)
    inside = _hull_pairs_equal(lqro_mod, recs, rrecs, "qhull")
    assert inside.sum() > 0
    assert np.array_equal(newv.view(np.uint64), rv.view(np.uint64))
