"""The boundary compiled from C++: tests/cpp/lqro_sim_main.cpp drives the
reference's agent loop (LQRObstacles.cpp:1391-1446) through the header-only
include/lqro_sim.hpp over lqro.h, built with plain g++ against liblqro.so
(__graft_entry__.build_cpp_demo, as INTEGRATION.md §1).  On the GPU its newV
must equal the oracle's step bit for bit and its agent update the oracle's
within the dynamics tolerance of tests/test_gpu_dyn.py; on the CPU the
binary must link and fail loudly (no gfx950 device), not fall back."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

DEMO = os.path.join(ROOT, "tests", "cpp", "lqro_sim_main")


@pytest.fixture(scope="module")
def demo(lqro_mod):
    if not os.path.exists(DEMO):
        import __graft_entry__ as ge
        ge.build_cpp_demo()
    return DEMO


def _write_input(path, x, vg, pg, H, NP, steps, seed):
    N = x.shape[0]
    with open(path, "wb") as f:
        np.array([N, H, NP, steps], np.int32).tofile(f)
        np.array([seed], np.uint32).tofile(f)
        for a in (x, vg, pg):
            np.ascontiguousarray(a, np.float64).tofile(f)


def test_cpp_consumer_links_and_fails_loudly_without_gpu(demo, tmp_path):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present (the -m gpu test covers the run)")
    x = np.zeros((4, 16))
    _write_input(tmp_path / "in.bin", x, np.zeros((4, 3)), np.zeros((4, 3)), 10, 20, 1, 1)
    r = subprocess.run([demo, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 1 and "no gfx950 device" in r.stderr, r.stderr


@pytest.mark.gpu
def test_cpp_consumer_matches_oracle(demo, lqro_mod, oracle, tmp_path):
    N, H, NP, steps, seed = 64, 50, 100, 2, 7
    x, vg = lqro_mod.synthetic_swarm(N)
    pg = -x[:, :3]
    _write_input(tmp_path / "in.bin", x, vg, pg, H, NP, steps, seed)
    r = subprocess.run([demo, str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = np.fromfile(tmp_path / "out.bin", np.float64).reshape(steps, -1)
    g = dict(oracle.synthesize(), l=np.zeros(4))
    T, NCF = oracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = oracle.sphere(NP)
    ref = lqro_mod.agent_states(x, p_goal=pg)
    ref["vgoal"][:] = vg
    sd = seed
    # lqro::Simulator takes lqro_config_default: the reference's own hull rule
    oracle.set_hull_rule(1, round16=True)
    oracle.carry_normal(np.zeros(3))
    try:
        for t in range(steps):
            newv = out[t, :N * 3].reshape(N, 3)
            xs = out[t, N * 3:].reshape(N, 16)
            rv, rr = oracle.step(T, NCF, S, ref["x"], ref["vgoal"], threads=8)
            if t == 0:
                assert np.array_equal(newv.view(np.uint64), rv.view(np.uint64))
            else:   # x went through one GPU dynamics step (libm last-bit differences)
                np.testing.assert_allclose(newv, rv, rtol=1e-5, atol=1e-6)
            ref["vgoal"][:] = rv
            nrm, sd = lqro_mod.normals(sd, N * lqro_mod.NORMALS_PER_AGENT)
            oracle.agent_step(ref, g, nrm)
            np.testing.assert_allclose(xs, ref["x"], rtol=1e-7, atol=1e-9)
    finally:
        oracle.set_hull_rule(0)
