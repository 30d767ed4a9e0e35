"""The oracle against the reference's own functions, live (CPU).

oracle/_ref/libref.so is the reference's per-pair path compiled from
/root/reference by oracle/Makefile (see oracle/ref_harness.cpp).  These tests
draw fresh random inputs — beyond the committed golden fixtures — and
require bit-identical results.  Skipped where the reference build is absent.
"""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def ref(oracle):
    r = oracle.reflib()
    if r is None:
        pytest.skip("oracle/_ref/libref.so not available (no /root/reference)")
    r.ref_pair.restype = C.c_int
    return r


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _bits(a):
    a = np.atleast_1d(np.asarray(a))
    return a.view(np.uint8)


@pytest.mark.parametrize("seed,box,H", [(101, 3.0, 30), (102, 5.0, 45), (103, None, 60)])
def test_pairs_random_swarms(oracle, ref, lqro_mod, seed, box, H):
    g = oracle.synthesize()
    N, NP = 10, 100
    x, _ = lqro_mod.synthetic_swarm(N, seed=seed, box=box)
    T, NCF = oracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = oracle.sphere(NP)
    idx = np.zeros(H * NP, np.int32)
    pts = np.zeros((H * NP, 3))
    for i in range(N):
        for j in range(N):
            if i == j:
                continue
            n = C.c_int(0)
            dist = np.zeros(1)
            nrm, wv, wh = np.zeros(3), np.zeros(3), np.zeros(3)
            pl = np.zeros(6, np.float32)
            xi, xj = np.ascontiguousarray(x[i]), np.ascontiguousarray(x[j])
            st = ref.ref_pair(NP, H, 4, C.c_double(30.0), _p(g["A"]), _p(g["B"]), _p(g["L"]),
                              _p(g["E"]), _p(xi), _p(xj), C.byref(n), _p(idx), _p(pts),
                              _p(dist), _p(nrm), _p(wv), _p(wh), _p(pl))
            rec, oidx, opts = oracle.pair(T, NCF, S, xi, xj, i, j, want_points=True)
            k = n.value
            assert rec["n_reach"] == k
            assert np.array_equal(oidx, idx[:k])
            assert np.array_equal(_bits(opts), _bits(pts[:k]))
            assert bool(rec["flags"] & 2) == (st == 1)
            if st == 0:
                assert np.array_equal(_bits(rec["dist"]), _bits(dist[0]))
                assert np.array_equal(_bits(rec["normal"]), _bits(nrm))
                got = np.concatenate([rec["plane_point"], rec["plane_normal"]]).astype(np.float32)
                assert np.array_equal(_bits(got), _bits(pl))


def test_gjk_random_clouds(oracle, ref):
    """gjk_distance (GJK:296-501) on random point clouds, point inside and
    outside: squared distance and both witnesses bit-identical."""
    rng = np.random.default_rng(7)
    ref.ref_gjk.restype = C.c_double
    lib = oracle.lib()
    for t in range(300):
        n = int(rng.integers(5, 400))
        pts = np.ascontiguousarray(rng.normal(size=(n, 3)) * rng.uniform(0.1, 10.0, size=3))
        v = np.ascontiguousarray(rng.normal(size=3) * (0.3 if t % 2 else 6.0))
        w1r, w2r = np.zeros(3), np.zeros(3)
        dr = ref.ref_gjk(n, _p(pts), _p(v), _p(w1r), _p(w2r))
        w1o, w2o = np.zeros(3), np.zeros(3)
        it, sn, bk = C.c_int(0), C.c_int(0), C.c_int(0)
        simplex = np.zeros(4, np.int32)
        do = lib.orc_gjk(_p(v), n, _p(pts), _p(w1o), _p(w2o), C.byref(it), C.byref(sn),
                         _p(simplex), C.byref(bk))
        assert np.array_equal(_bits(do), _bits(dr)), t
        assert np.array_equal(_bits(w1o), _bits(w1r)) and np.array_equal(_bits(w2o), _bits(w2r)), t


def test_newv_random(oracle, ref):
    from lp_cases import random_cases
    cases, goals = random_cases(150, seed=11)
    for c, v in zip(cases, goals):
        c = np.ascontiguousarray(c, np.float32)
        v = np.ascontiguousarray(v, np.float64)
        out = np.zeros(3)
        ref.ref_newv(c.shape[0], _p(c), _p(v), _p(out))
        assert np.array_equal(_bits(oracle.newv(c, v)), _bits(out))


def test_inverse_matches_reference(oracle, ref):
    """operator! (MAT:603-671) via the gain synthesis: covered bit-exactly by
    test_oracle_golden.test_gains_bit_exact; here the 3x3 inverse the tables
    use (T_k = (C G_k)^-1) on random matrices."""
    rng = np.random.default_rng(3)
    lib = oracle.lib()
    if not hasattr(lib, "orc_inverse3"):
        pytest.skip("oracle does not export orc_inverse3")
    for _ in range(200):
        m = np.ascontiguousarray(rng.normal(size=(3, 3)))
        a, b = np.zeros(9), np.zeros(9)
        ref.ref_inverse3(_p(m), _p(a))
        lib.orc_inverse3(_p(m), _p(b))
        assert np.array_equal(_bits(a), _bits(b))
    for _ in range(100):
        m = np.ascontiguousarray(rng.normal(size=(4, 4)))
        a, b = np.zeros(16), np.zeros(16)
        ref.ref_inverse4(_p(m), _p(a))
        lib.orc_inverse4(_p(m), _p(b))
        assert np.array_equal(_bits(a), _bits(b))
