"""Opt-in neighbour culling (RVO2 computeNeighbors /
insertAgentNeighbor, AGT:74-81,153-174).  The oracle's selection against a
brute-force restatement (CPU), then the GPU step with culling against the
oracle step with culling (bit-exact records and newV)."""
import numpy as np
import pytest


def _brute(x, i, r, k):
    d = x[i, :3] - x[:, :3]   # the kernels' op order: dx*dx + dy*dy + dz*dz
    d2 = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2]
    cand = [(d2[j], j) for j in range(len(x)) if j != i and d2[j] < r * r]
    keep = sorted(cand)[:k]
    sel = np.zeros(len(x), np.uint8)
    for _, j in keep:
        sel[j] = 1
    return sel


@pytest.mark.parametrize("seed,k,r", [(1, 4, 2.0), (2, 10, 3.0), (3, 100, 1.5), (4, 3, 50.0)])
def test_oracle_selection(oracle, lqro_mod, seed, k, r):
    x, _ = lqro_mod.synthetic_swarm(40, seed=seed, box=4.0)
    for i in range(0, 40, 7):
        assert np.array_equal(oracle.neighbors(x, i, r, k), _brute(x, i, r, k))


def test_oracle_selection_ties(oracle):
    """Equal distances: the lower j is kept (RVO2 keeps the earlier-visited)."""
    x = np.zeros((7, 16))
    for j, p in enumerate([(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (-1, 0, 0), (2, 0, 0), (0, -1, 0)]):
        x[j, :3] = p
    sel = oracle.neighbors(x, 0, 10.0, 3)
    assert sel.tolist() == [0, 1, 1, 1, 0, 0, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("k,r,box", [(6, 2.5, 3.0), (1, 1.0, 3.0), (500, 1000.0, 3.0), (8, 3.0, 1.6)])
def test_gpu_step_with_culling(lqro_mod, oracle, gains, k, r, box):
    """box 1.6: a dense swarm, so neighbour pairs reach the in-kernel hull
    (slot -> neighbour mapping in k_hull)."""
    N, H, NP = 48, 40, 50
    x, vg = lqro_mod.synthetic_swarm(N, seed=17, box=box)
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    S = oracle.sphere(NP)
    oracle.set_neighbors(r, k)
    try:
        rv, rrecs = oracle.step(T, NCF, S, x, vg)
    finally:
        oracle.set_neighbors(0.0, 0)
    ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, flags=lqro_mod.LQRO_FLAG_RECORDS))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    ctx.set_neighbors(r, k)
    newv = ctx.step(x, vg)
    recs = ctx.records()
    K = min(k, N - 1)
    assert recs.shape[0] == N * K
    kept = rrecs["n_reach"] >= 0
    assert ctx.stats()["pairs"] == int(kept.sum())
    rr = rrecs.reshape(N, N - 1)
    gr = recs.reshape(N, K)
    for i in range(N):   # row i: its neighbours in ascending j, then empty slots
        ref_row = rr[i][rr[i]["n_reach"] >= 0]
        c = len(ref_row)
        assert c <= K and np.all(gr[i][c:]["n_reach"] == -1) and np.all(gr[i][c:]["j"] == -1)
        g = gr[i][:c]
        for f in ("i", "j", "n_reach", "flags", "gjk_iters", "simplex_n", "reach_hash"):
            a = g[f] & ~lqro_mod.REC_LOCAL if f == "flags" else g[f]   # the oracle has no local hull
            assert np.array_equal(a, ref_row[f]), (i, f)
        for f in ("plane_point", "plane_normal"):
            assert np.array_equal(g[f].view(np.uint32), ref_row[f].view(np.uint32)), (i, f)
        ins = (g["flags"] & lqro_mod.REC_INSIDE) != 0
        assert np.array_equal(g["facet"][ins], ref_row["facet"][ins]), i
    if box < 2:
        assert int(((recs["flags"] & lqro_mod.REC_INSIDE) != 0).sum()) > 0
    np.testing.assert_array_equal(newv, rv)
    # all pairs again
    ctx.set_neighbors(0.0, 0)
    ctx.step(x, vg)
    assert ctx.stats()["pairs"] == N * (N - 1)


@pytest.mark.gpu
def test_gpu_culling_many_candidates(lqro_mod, oracle, gains):
    """More agents within the radius than k_nbr's LDS candidate list holds
    (1,024): the selection falls back to scanning global memory per round."""
    N, H, NP, k, r = 1100, 20, 50, 3, 1.0e4
    x, vg = lqro_mod.synthetic_swarm(N, seed=19)
    T, NCF = oracle.tables(gains["A"], gains["B"], gains["L"], gains["E"], H)
    S = oracle.sphere(NP)
    oracle.set_neighbors(r, k)
    try:
        rv, rrecs = oracle.step(T, NCF, S, x, vg, rows=(0, 24))
    finally:
        oracle.set_neighbors(0.0, 0)
    ctx = lqro_mod.Context(lqro_mod.config(N, H, NP, flags=lqro_mod.LQRO_FLAG_RECORDS,
                                           row_begin=0, row_end=24))
    ctx.set_gains(gains["A"], gains["B"], gains["L"], gains["E"])
    ctx.set_neighbors(r, k)
    newv = ctx.step(x, vg)
    gr = ctx.records().reshape(24, k)
    rr = rrecs.reshape(24, N - 1)
    for i in range(24):
        ref_row = rr[i][rr[i]["n_reach"] >= 0]
        assert len(ref_row) == k
        for f in ("j", "n_reach", "flags", "reach_hash"):
            a = gr[i][f] & ~lqro_mod.REC_LOCAL if f == "flags" else gr[i][f]
            assert np.array_equal(a, ref_row[f]), (i, f)
    np.testing.assert_array_equal(newv[:24], rv[:24])
