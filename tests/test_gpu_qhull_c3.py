"""The default rule (LQRO_FLAG_QHULL_ORDER: Qhull's build order, the planes
read back at 16 digits, first Fv vertex, strict '<', the loop-carried normal;
LQRObstacles.cpp:867-969, 1385) pinned at the sizes where the canonical rule
was pinned:

- C3 (1024 agents, H = 100: 1,047,552 pairs): every record and every row's
  newV bit for bit against the oracle in set_hull_rule(1), in every schedule
  the step can take there — the default (hot launch, side builds, early LP:
  the row-counting protocol of lqro_hull.hpp hull_row_done that closes a row
  and runs its LP inside k_qhull; from the third step the speculative builds:
  the last step's inside-hull pairs queued for k_qhull at the step's start,
  built at once, committed when the main stream's hot launch finds them
  inside, dropped when it does not), LQRO_HOT_SPEC=0 (the split hot launch:
  those pairs evaluated alone on the side stream first), LQRO_EARLY_LP=0,
  LQRO_HOT_SPLIT=0, LQRO_QSIDE=1 (side workers sweep rows after their
  builds), LQRO_QHULL_SPARE=0 (one side CU per last-step inside pair: a pair
  new this step waits for the first build to end), LQRO_HOT=0 (plain),
  LQRO_QHULL_BALANCE=0 (round 5's side width, one CU per expected build) and
  LQRO_QHULL_INLINE_BIG=0 (capped builds to k_qhull_big after the sweep);
- C5 (16384 agents, X = 12, H = 200, per-agent gains): the 8-way shard
  [0, 2048) in Qhull order on the GPU, 32 rows' newV against the oracle, each
  entered with the loop-carried normal the shard's rows before it left (the
  row-normal table of lqro_step_device_begin);
- qconvex's merged winners (tests/golden/qhull_merge.npz, live Qhull): the
  pairs are flagged LQRO_REC_QHMERGE_WIN, as the oracle flags them;
- the per-build timing records (lqro_get_hull_builds)."""
import numpy as np
import pytest

from conftest import GOLDEN
from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu

QFIELDS = ("n_reach", "reach_hash", "flags", "facet", "n_facets", "dist", "normal", "plane_point", "plane_normal",
           "gjk_iters", "simplex_n", "simplex", "wpt_vrel", "wpt_hull")


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint8) if a.dtype.kind == "f" else a


@pytest.fixture(scope="module")
def c3_oracle(lqro_mod, oracle, gains):
    N, H = 1024, 100
    x, vg = lqro_mod.synthetic_swarm(N)
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    oracle.set_hull_rule(1, round16=True)
    oracle.carry_normal(np.zeros(3))
    try:
        rv, rr = oracle.step(T, NCF, oracle.sphere(100), x, vg, threads=16)
        carry = oracle.carry_normal()
    finally:
        oracle.set_hull_rule(0)
    return x, vg, rv, rr, carry


@pytest.mark.parametrize("sched", ["default", "no_spec", "spare0", "early_lp_off", "no_split", "qside", "plain",
                                   "balance_off", "inline_big", "qflags0"])
def test_qhull_order_c3_full_step(lqro_mod, gains, monkeypatch, c3_oracle, sched):
    x, vg, rv, rr, carry = c3_oracle
    env = {"default": {}, "no_spec": {"LQRO_HOT_SPEC": "0"}, "spare0": {"LQRO_QHULL_SPARE": "0"},
           "early_lp_off": {"LQRO_EARLY_LP": "0"},
           "no_split": {"LQRO_HOT_SPLIT": "0"}, "qside": {"LQRO_QSIDE": "1"}, "plain": {"LQRO_HOT": "0"},
           "balance_off": {"LQRO_QHULL_BALANCE": "0"}, "inline_big": {"LQRO_QHULL_INLINE_BIG": "0"},
           # (k_qhull without its round-6 helpers, lane state, queue pre-scan and bucketed emit)
           "qflags0": {"LQRO_QHULL_FLAGS": "0"}}[sched]
    for k in ("LQRO_EARLY_LP", "LQRO_QSIDE", "LQRO_HOT", "LQRO_LOCAL_HULL", "LQRO_SIDE_HULL_CUS", "LQRO_HOT_SPLIT",
              "LQRO_HOT_SPEC", "LQRO_QHULL_SPARE", "LQRO_QHULL_BALANCE", "LQRO_QHULL_INLINE_BIG", "LQRO_QHULL_FLAGS"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    N = x.shape[0]
    ctx = lqro_mod.Context(lqro_mod.config(N, 100, 100,
                                           flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    try:
        # three steps, each entered with the normal 0 (as the oracle's): the
        # schedule adapts to the inside-hull count of the step two before, so
        # the third is the steady state
        for t in range(3):
            ctx.carry_normal(np.zeros(3))
            v = ctx.step(x, vg)
            r = ctx.records()
            st = ctx.stats()
            assert st["hull_fail"] == 0 and st["qhull_timeouts"] == 0
            _compare(r, rr)
            ins = (rr["flags"] & lqro_mod.REC_INSIDE) != 0
            assert ins.sum() > 100
            for f in QFIELDS:
                a, b = r[f], rr[f]
                if f == "flags":
                    a = a & ~lqro_mod.REC_LOCAL
                assert np.array_equal(_bits(a), _bits(b)), (sched, t, f)
            assert np.array_equal(v.view(np.uint64), rv.view(np.uint64)), (sched, t)
            assert np.array_equal(ctx.carry_normal(), carry)
    finally:
        ctx.close()


@pytest.fixture(scope="module")
def c3_oracle_moved(lqro_mod, oracle, gains, c3_oracle):
    """The C3 swarm 1 s later (positions advanced by their velocities): its
    inside-hull pairs differ from the first swarm's both ways."""
    x, vg = c3_oracle[0], c3_oracle[1]
    x1 = x.copy()
    x1[:, 0:3] += 1.0 * x[:, 3:6]
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], 100)
    oracle.set_hull_rule(1, round16=True)
    oracle.carry_normal(np.zeros(3))
    try:
        rv, rr = oracle.step(T, NCF, oracle.sphere(100), x1, vg, threads=16)
        carry = oracle.carry_normal()
    finally:
        oracle.set_hull_rule(0)
    return x1, rv, rr, carry


@pytest.mark.parametrize("sched", ["default", "no_spec", "spare0", "side_pct50"])
def test_speculative_builds_moving_swarm(lqro_mod, gains, monkeypatch, c3_oracle, c3_oracle_moved, sched):
    """Speculative builds when the inside-hull set changes between steps: the
    swarm at x0, x0, x1, x0 — the third step's builds were queued for x0's
    inside pairs (those not inside at x1 are dropped, x1's new ones queued by
    their evaluation), the fourth's for x1's.  Each step bit for bit against
    the oracle at its own state, in every schedule that carries state across
    steps (the last step's inside-hull list d_prevq, the hot marks, k_prio_save's
    order): the default, the split hot launch without speculative builds
    (LQRO_HOT_SPEC=0: at the fourth step a pair inside at x0 but not at x1
    must not keep the third step's "listed" mark), no spare CU and half a side."""
    x0, vg, rv0, rr0, carry0 = c3_oracle
    x1, rv1, rr1, carry1 = c3_oracle_moved
    for k in ("LQRO_EARLY_LP", "LQRO_QSIDE", "LQRO_HOT", "LQRO_LOCAL_HULL", "LQRO_SIDE_HULL_CUS", "LQRO_HOT_SPLIT",
              "LQRO_HOT_SPEC", "LQRO_QHULL_SPARE", "LQRO_QHULL_SIDE_PCT"):
        monkeypatch.delenv(k, raising=False)
    env = {"default": {}, "no_spec": {"LQRO_HOT_SPEC": "0"}, "spare0": {"LQRO_QHULL_SPARE": "0"},
           "side_pct50": {"LQRO_QHULL_SIDE_PCT": "50"}}[sched]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    in0 = (rr0["flags"] & lqro_mod.REC_INSIDE) != 0
    in1 = (rr1["flags"] & lqro_mod.REC_INSIDE) != 0
    assert (in0 & ~in1).sum() > 0 and (in1 & ~in0).sum() > 0, ((in0 & ~in1).sum(), (in1 & ~in0).sum())
    N = x0.shape[0]
    ctx = lqro_mod.Context(lqro_mod.config(N, 100, 100,
                                           flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    try:
        for t, (x, rv, rr, carry) in enumerate([(x0, rv0, rr0, carry0), (x0, rv0, rr0, carry0),
                                                (x1, rv1, rr1, carry1), (x0, rv0, rr0, carry0)]):
            ctx.carry_normal(np.zeros(3))
            v = ctx.step(x, vg)
            r = ctx.records()
            st = ctx.stats()
            assert st["hull_fail"] == 0 and st["qhull_timeouts"] == 0
            _compare(r, rr)
            for f in QFIELDS:
                a, b = r[f], rr[f]
                if f == "flags":
                    a = a & ~lqro_mod.REC_LOCAL
                assert np.array_equal(_bits(a), _bits(b)), (sched, t, f)
            assert np.array_equal(v.view(np.uint64), rv.view(np.uint64)), (sched, t)
            assert np.array_equal(ctx.carry_normal(), carry), (sched, t)
    finally:
        ctx.close()


def test_c5_qhull_order_rows(lqro_mod, oracle):
    """C5's first 8-way shard in Qhull order: 32 rows spread over it against
    the oracle, bit for bit, each row entered with the normal the rows before
    it left (the row-normal table: a facet-0 pair at the top of a row takes
    the previous rows' last normal, LQRO:1385)."""
    from test_gpu_dyn import _Hip   # device buffers through liblqro's own HIP runtime
    N, H, NP, X = 16384, 200, 100, 12
    rows = (0, 2048)
    models = lqro_mod.perturbed_models(N)
    g = lqro_mod.synthesize_gains_batch(models, x_dim=X)
    g0 = lqro_mod.synthesize_gains(x_dim=X)
    x, vg = lqro_mod.synthetic_swarm(N, x_dim=X)
    ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, x_dim=X, row_begin=rows[0], row_end=rows[1],
                                           flags=lqro_mod.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(g0["A"], g0["B"], g["L"], g["E"], per_agent=True)
    hip = _Hip()
    zt, zv = np.zeros((N, 4)), np.zeros((N, 3))
    d_x, d_vg, d_tab, d_nv = hip.put(x), hip.put(vg), hip.put(zt), hip.put(zv)
    ctx.step_device_begin(d_x, d_vg, d_tab, 0)
    ctx.step_device_end(d_tab, d_nv, 0)
    hip.sync()
    st = ctx.stats()
    ctx.close()
    newv, tab = hip.get(d_nv, zv), hip.get(d_tab, zt)
    assert st["hull_fail"] == 0 and st["inside"] > 500, st
    own = newv[rows[0]:rows[1]]
    assert np.isfinite(own).all()
    S = oracle.sphere(NP)
    oracle.set_hull_rule(1, round16=True)
    T = np.zeros((N, H, 9))
    NCF = np.zeros((N, H, 3, X))
    try:
        for r in range(7, 2048, 64):
            prev = [q for q in range(rows[0], r) if tab[q, 3] != 0]
            carry = tab[prev[-1], :3] if prev else np.zeros(3)
            T[r], NCF[r] = oracle.tables(g0["A"], g0["B"], g["L"][r], g["E"][r], H, X=X)
            oracle.carry_normal(carry)
            rv, _ = oracle.step(T, NCF, S, x, vg, rows=(r, r + 1), per_agent=True, threads=16, records=False)
            assert np.array_equal(newv[r].view(np.uint64), rv[r].view(np.uint64)), r
            if tab[r, 3] != 0:
                assert np.array_equal(oracle.carry_normal(), tab[r, :3]), r
    finally:
        oracle.set_hull_rule(0)


def test_merged_winners_are_flagged(lqro_mod, oracle, gains):
    """Inputs where qconvex's pre-merge joins the winning facet (coplanar
    cube faces, a flattened cap; tests/golden/make_golden_merge.py over live
    Qhull): k_qhull (built merge-free) flags each LQRO_REC_QHMERGE and
    LQRO_REC_QHMERGE_WIN, exactly as the oracle does, its selection equals
    the oracle's merge-free one bit for bit, and the C-ABI reports the pair
    loudly (LQRO_E_QHMERGE, lqro_step's rule) — never the silent LQRO_OK; the
    reference's own fixture (no merge) reports LQRO_OK."""
    d = np.load(f"{GOLDEN}/qhull_merge.npz")
    ctx = lqro_mod.Context(lqro_mod.config(2, 100, 100))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    oracle.set_hull_rule(1, round16=True)
    try:
        for c in ("cube_top", "cube_side", "capped"):
            assert d[f"{c}_expect"][1] == 1, c           # qconvex's winner is a merged facet
            rec, st = ctx.debug_qhull(d[f"{c}_rounded"], d[f"{c}_pts"], d[f"{c}_vrel"])
            assert ctx.debug_status == lqro_mod.LQRO_E_QHMERGE, (c, ctx.debug_status)
            nf, dist, nrm, fac, qst = oracle.hull_branch_ref(d[f"{c}_pts"], d[f"{c}_vrel"])
            assert qst & 0x10000, c
            assert rec["flags"] & lqro_mod.REC_QHMERGE and rec["flags"] & lqro_mod.REC_QHMERGE_WIN, (c, rec["flags"])
            assert rec["n_facets"] == nf and list(rec["facet"]) == list(fac) and rec["dist"] == dist, c
            if nrm is not None:
                assert np.array_equal(rec["normal"], nrm), c
        from test_oracle_golden import _qhull_fixture
        pts, _, _ = _qhull_fixture()
        pts = np.ascontiguousarray(pts, np.float64)
        rec, st = ctx.debug_qhull(pts, pts, pts.mean(0))
        assert ctx.debug_status == lqro_mod.LQRO_OK and not rec["flags"] & lqro_mod.REC_QHMERGE_WIN
    finally:
        oracle.set_hull_rule(0)
        ctx.close()


def test_hull_build_records(lqro_mod, gains):
    """lqro_get_hull_builds: one record per inside-hull pair of the step,
    naming the pair, with its insertions, facets and a positive duration on
    the 100 MHz clock; the counts agree with the pair records."""
    N = 256
    x, vg = lqro_mod.synthetic_swarm(N, box=12.0, seed=3)
    ctx = lqro_mod.Context(lqro_mod.config(N, 100, 100,
                                           flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    try:
        ctx.step(x, vg)
        r = ctx.records()
        b = ctx.hull_builds()
    finally:
        ctx.close()
    ins = r[(r["flags"] & lqro_mod.REC_INSIDE) != 0]
    assert len(ins) > 10
    done = b[b["kernel"] != 2]
    assert len(done) == len(ins)
    assert sorted(zip(done["i"].tolist(), done["j"].tolist())) == sorted(zip(ins["i"].tolist(), ins["j"].tolist()))
    assert (done["insertions"] > 4).all() and (done["facet_slots"] > done["insertions"]).all()
    assert (done["t_end"] > done["t_start"]).all()
    by = {(int(q["i"]), int(q["j"])): q for q in ins}
    for q in done:
        assert q["n_points"] == by[(int(q["i"]), int(q["j"]))]["n_reach"]


def test_recycled_device_memory(lqro_mod, gains, monkeypatch, c3_oracle):
    """A context on device memory that held other data: the hot marks start
    at 0 whatever the allocator hands back (k_prio keeps a mark of 2, k_prio_prev's
    "listed", so recycled bytes of 2 made the first split step skip those
    pairs).  1.3 GiB are filled with 2s and freed first; the third step (the
    first with the split hot launch) bit for bit against the oracle."""
    from test_gpu_dyn import _Hip
    import ctypes as C
    x, vg, rv, rr, carry = c3_oracle
    for k in ("LQRO_EARLY_LP", "LQRO_QSIDE", "LQRO_HOT", "LQRO_LOCAL_HULL", "LQRO_SIDE_HULL_CUS", "LQRO_HOT_SPLIT",
              "LQRO_HOT_SPEC", "LQRO_QHULL_SPARE", "LQRO_QHULL_BALANCE", "LQRO_QHULL_INLINE_BIG"):
        monkeypatch.delenv(k, raising=False)
    hip = _Hip()
    blocks = []
    slots = 1024 * 1023
    for size in [32 << 20] * 32 + [slots] * 256:   # (large blocks, and blocks of the marks' own size)
        p = C.c_void_p()
        if hip.h.hipMalloc(C.byref(p), C.c_size_t(size)) != 0:
            break
        assert hip.h.hipMemset(p, 2, C.c_size_t(size)) == 0
        blocks.append(p)
    assert hip.h.hipDeviceSynchronize() == 0
    for p in blocks:
        assert hip.h.hipFree(p) == 0
    ctx = lqro_mod.Context(lqro_mod.config(1024, 100, 100,
                                           flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    try:
        for t in range(3):
            ctx.carry_normal(np.zeros(3))
            v = ctx.step(x, vg)
        r = ctx.records()
        _compare(r, rr)
        assert np.array_equal(v.view(np.uint64), rv.view(np.uint64))
    finally:
        ctx.close()
