"""The oracle's per-agent step after the pair loop (LQRO:1437-1446) against
the reference: the committed fixture tests/golden/dyn.npz (any machine) and
the reference's own functions live where oracle/_ref/libref.so exists — all
bit-exact (both are gcc/glibc builds).  jacobi and sampleGaussian, which the
reference cannot build here (MSVC _hypot), are pinned by their properties and
through kalmanFilter1."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLDEN
from dyn_cases import random_agent_cases


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(os.path.join(GOLDEN, "dyn.npz")))


@pytest.fixture(scope="module")
def gains(oracle, gold):
    g = oracle.synthesize()
    g["l"] = gold["l"]
    return g


def _model(oracle):
    m = oracle.Model()
    oracle.lib().orc_model_default(C.byref(m))
    return m


def _run_oracle(oracle, g, cs):
    o = oracle.lib()
    n = cs["x"].shape[0]
    m = _model(oracle)
    M, N = 1e-9 * np.eye(16), 1e-9 * np.eye(6)
    u, v = np.zeros((n, 4)), np.zeros((n, 3))
    k1 = {k: cs[k].copy() for k in ("x", "rot", "P")}
    k2 = {k: cs[k].copy() for k in ("x", "rot", "P")}
    for a in range(n):
        o.orc_control_velocity(_p(cs["x"][a]), _p(cs["rot"][a]), _p(cs["vgoal"][a]),
                               _p(cs["u_goal"][a]), _p(g["L"]), _p(g["E"]), _p(g["l"]), _p(u[a]))
        o.orc_control_position(_p(cs["x"][a]), _p(cs["rot"][a]), _p(cs["p_goal"][a]),
                               _p(cs["u_goal"][a]), _p(g["Lh"]), _p(g["Eh"]), _p(v[a]))
        o.orc_kalman1(C.byref(m), _p(k1["x"][a]), _p(k1["rot"][a]), _p(u[a]), _p(M), _p(k1["P"][a]))
        o.orc_kalman2(C.byref(m), _p(k2["x"][a]), _p(k2["rot"][a]), _p(cs["z"][a]), _p(N),
                      _p(k2["P"][a]))
    return u, v, k1, k2


def _same(a, b):
    assert a.shape == b.shape
    assert np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64)), \
        f"max |diff| {np.abs(a - b).max()}"


def test_against_golden(oracle, gains, gold):
    cs = {k[3:]: gold[k].copy() for k in gold if k.startswith("in_")}
    u, v, k1, k2 = _run_oracle(oracle, gains, cs)
    _same(u, gold["u"])
    _same(v, gold["v"])
    for k in ("x", "rot", "P"):
        _same(k1[k], gold["k1_" + k])
        _same(k2[k], gold["k2_" + k])


def test_against_reference_live(oracle, gains):
    r = oracle.reflib()
    if r is None:
        pytest.skip("oracle/_ref/libref.so not available (no /root/reference)")
    cs = random_agent_cases(40, seed=777)
    g = dict(gains)
    g["l"] = np.array([0.01, -0.02, 0.03, -0.04])   # exercise the + l term
    u, v, k1, k2 = _run_oracle(oracle, g, cs)
    l_ref = np.zeros(4)
    r.ref_gain_l(_p(l_ref))
    _same(l_ref, gains["l"])
    for a in range(cs["x"].shape[0]):
        ur, vr = np.zeros(4), np.zeros(3)
        r.ref_control_velocity(_p(cs["x"][a]), _p(cs["rot"][a]), _p(cs["vgoal"][a]),
                               _p(cs["u_goal"][a]), _p(g["L"]), _p(g["E"]), _p(g["l"]), _p(ur))
        r.ref_control_position(_p(cs["x"][a]), _p(cs["rot"][a]), _p(cs["p_goal"][a]),
                               _p(cs["u_goal"][a]), _p(g["Lh"]), _p(g["Eh"]), _p(vr))
        _same(u[a], ur)
        _same(v[a], vr)
        for kk, fn, arg in ((k1, r.ref_kalman1, u[a]), (k2, r.ref_kalman2, cs["z"][a])):
            xs, rs, ps = cs["x"][a].copy(), cs["rot"][a].copy(), cs["P"][a].copy()
            fn(_p(xs), _p(rs), _p(arg), _p(ps))
            _same(kk["x"][a], xs)
            _same(kk["rot"][a], rs)
            _same(kk["P"][a], ps)


@pytest.mark.parametrize("n,seed", [(16, 1), (6, 2), (3, 3)])
@pytest.mark.parametrize("scale", [1.0, 1e-9])
def test_jacobi_properties(oracle, n, seed, scale):
    """Rotations run until every off-diagonal is <= DBL_EPSILON in absolute
    value (MAT:701): at unit scale that is a full eigendecomposition; at the
    noise covariances' scale (~1e-9) it stops almost at once, as in the
    reference, and the dropped off-diagonals are each <= DBL_EPSILON."""
    rng = np.random.default_rng(seed)
    B = rng.normal(size=(n, n))
    m = (B @ B.T + np.eye(n)) * scale
    V, D = oracle.jacobi(m)
    eps = np.finfo(float).eps
    assert np.array_equal(D, np.diag(np.diag(D)))
    np.testing.assert_allclose(V @ V.T, np.eye(n), atol=1e-13)
    np.testing.assert_allclose(V @ D @ V.T, m, atol=n * eps + 1e-13 * scale, rtol=0)
    if scale == 1.0:
        np.testing.assert_allclose(np.sort(np.diag(D)), np.linalg.eigvalsh(m), rtol=1e-12)


def test_propagate_noise_free_is_kalman1(oracle, gains):
    """propagate with zero draws = kalmanFilter1's state update, bit for bit
    (sampleGaussian(0, MM) contributes exact zeros)."""
    cs = random_agent_cases(8, seed=11, rot_err=False)
    o = oracle.lib()
    m = _model(oracle)
    M = 1e-9 * np.eye(16)
    z16 = np.zeros(16)
    for a in range(8):
        u = cs["u_goal"][a] + 0.05
        x1, r1, p1 = cs["x"][a].copy(), cs["rot"][a].copy(), cs["P"][a].copy()
        x2, r2 = cs["x"][a].copy(), cs["rot"][a].copy()
        o.orc_kalman1(C.byref(m), _p(x1), _p(r1), _p(u), _p(M), _p(p1))
        o.orc_propagate(C.byref(m), _p(x2), _p(r2), _p(u), _p(M), _p(z16))
        _same(x1, x2)
        _same(r1, r2)


def test_msvc_normals_known_answer(lqro_mod):
    """lqro_normals runs normal() (LQRO:340-350) over the MSVC rand() stream:
    srand(1) gives 41, 18467, 6334, 26500, ... (the CRT's documented LCG)."""
    seed = 1
    rands = []
    for _ in range(8):
        seed = (seed * 214013 + 2531011) & 0xFFFFFFFF
        rands.append((seed >> 16) & 0x7FFF)
    assert rands[:4] == [41, 18467, 6334, 26500]
    uni = [(rands[2 * k] * 32768 + rands[2 * k + 1]) / (32767 * 32769) for k in range(4)]
    u, v = 2 * uni[0] - 1, 2 * uni[1] - 1
    s = u * u + v * v
    if s == 0 or s > 1:
        u, v = 2 * uni[2] - 1, 2 * uni[3] - 1
        s = u * u + v * v
    draws, nxt = lqro_mod.normals(1, 20000)
    assert draws[0] == u * np.sqrt(-2 * np.log(s) / s)
    assert abs(draws.mean()) < 0.03 and abs(draws.std() - 1) < 0.03
    d2, _ = lqro_mod.normals(1, 20000)
    assert np.array_equal(draws, d2) and nxt != 1


def test_quat_from_rot(oracle, gold):
    """quatFromRot (stdafx.h:24-33), the orientation of visualize's keyframe:
    against the golden fixture and, where available, the live reference."""
    o = oracle.lib()
    qin = gold["quat_in"]
    got = np.zeros((qin.shape[0], 4))
    for a in range(qin.shape[0]):
        o.orc_quat_from_rot(_p(np.ascontiguousarray(qin[a])), _p(got[a]))
    _same(got, gold["quat_out"])
    r = oracle.reflib()
    if r is not None:
        rng = np.random.default_rng(5)
        from dyn_cases import rotation
        for _ in range(50):
            R = rotation(rng.normal(size=3) * rng.uniform(0, 3.14))
            q1, q2 = np.zeros(4), np.zeros(4)
            o.orc_quat_from_rot(_p(R), _p(q1))
            r.ref_quat_from_rot(_p(R), _p(q2))
            _same(q1, q2)
