"""The per-agent step after the pair loop on the GPU (lqro_dynamics_step,
k_dyn: findU, propagate, kalmanFilter1, the observation draw, kalmanFilter2,
findVGoal — LQRO:1437-1446) against the oracle's C
restatement (tests/test_oracle_dyn.py pins that to the reference).

Tolerance: the step calls libm on live values (tan in f, asin in the
controllers, atan2 in errFromRot, hypot in jacobi), where the device's and
glibc's results may differ in the last bit, so results are compared with a
relative tolerance of 1e-9 after one step and 1e-6 after a 30-step
trajectory (SURVEY §8c allows 1e-5 for fp64 outputs)."""
import ctypes as C

import numpy as np
import pytest

from dyn_cases import trajectory_start

pytestmark = pytest.mark.gpu

STATE = ("x", "rot", "x_true", "rot_true", "P", "vgoal")


def _gains(oracle, l=(0.01, -0.02, 0.03, -0.04)):
    g = oracle.synthesize()
    g["l"] = np.array(l, dtype=np.float64)
    return g


def _states(lqro_mod, n, seed):
    cs = trajectory_start(n, seed)
    st = lqro_mod.agent_states(cs["x"], p_goal=cs["p_goal"])
    st["rot"][:] = cs["rot"]
    st["rot_true"][:] = cs["rot"]
    st["P"][:] = cs["P"]
    st["vgoal"][:] = cs["vgoal"]
    return st


def _close(a, b, rtol, what):
    scale = np.maximum(np.abs(b), 1e-3 * np.abs(b).max() + 1e-300)
    err = (np.abs(a - b) / scale).max()
    assert err <= rtol, f"{what}: max rel err {err:.3e}"


def _compare(g, r, rtol):
    for k in STATE:
        _close(g[k], r[k], rtol, k)


def test_one_step(lqro_mod, oracle):
    n = 200
    g = _gains(oracle)
    st = _states(lqro_mod, n, seed=21)
    ref = {k: v.copy() for k, v in st.items()}
    nrm, _ = lqro_mod.normals(7, n * lqro_mod.NORMALS_PER_AGENT)
    kf = np.zeros((n, 8), np.float32)
    u = lqro_mod.dynamics_step(st, g, nrm, keyframes=kf, time=1.25)
    ur = oracle.agent_step(ref, g, nrm)
    # visualize's keyframe from the step's own xTrue / RotTrue, bit for bit
    assert np.array_equal(kf.view(np.uint32),
                          oracle.keyframes(1.25, st["x_true"], st["rot_true"]).view(np.uint32))
    _close(u, ur, 1e-9, "u")
    _compare(st, ref, 1e-9)
    assert np.all(st["x"][:, 6:9] == 0)     # rotation error reset into Rot
    np.testing.assert_allclose(np.einsum("nij,nkj->nik", st["rot"], st["rot"]),
                               np.tile(np.eye(3), (n, 1, 1)), atol=1e-12)


def test_trajectory(lqro_mod, oracle):
    """30 steps of the closed loop velocity -> position controller with the
    reference's noise stream (srand(1), agent order)."""
    n = 48
    g = _gains(oracle)
    st = _states(lqro_mod, n, seed=22)
    ref = {k: v.copy() for k, v in st.items()}
    seed = 1
    for t in range(30):
        nrm, seed = lqro_mod.normals(seed, n * lqro_mod.NORMALS_PER_AGENT)
        lqro_mod.dynamics_step(st, g, nrm)
        oracle.agent_step(ref, g, nrm)
    _compare(st, ref, 1e-6)
    # the agents head for their position goals
    assert np.all(np.isfinite(st["x"]))


def test_heterogeneous(lqro_mod, oracle):
    """Per-agent models and gains (C5-style swarm): lqro_synthesize_gains_batch
    feeds lqro_dynamics_step(per_agent_gains = 1)."""
    from test_gpu_synth import perturbed_models
    n = 64
    models = perturbed_models(lqro_mod, n, seed=5)
    gb = lqro_mod.synthesize_gains_batch(models)
    gb["l"] = np.random.default_rng(3).uniform(-0.02, 0.02, (n, 4))
    st = _states(lqro_mod, n, seed=23)
    ref = {k: v.copy() for k, v in st.items()}
    nrm, _ = lqro_mod.normals(99, n * lqro_mod.NORMALS_PER_AGENT)
    u = lqro_mod.dynamics_step(st, gb, nrm, models=models, per_agent=True)
    ur = oracle.agent_step(ref, gb, nrm, models=models, per_agent=True)
    _close(u, ur, 1e-9, "u")
    _compare(st, ref, 1e-9)


class _Hip:
    """Device buffers through the HIP runtime liblqro.so itself links
    (libamdhip64): torch's bundled runtime is not initialised in this process."""

    def __init__(self):
        # the copy liblqro.so loaded (a second HIP runtime in one process, e.g.
        # torch's bundled one, sees no device)
        path = "libamdhip64.so"
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line and "/opt/rocm" in line:
                    path = line.split()[-1]
                    break
        self.h = C.CDLL(path)
        self.ptrs = []

    def put(self, a: np.ndarray) -> int:
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        assert self.h.hipMalloc(C.byref(p), C.c_size_t(max(a.nbytes, 8))) == 0
        self.ptrs.append(p)
        assert self.h.hipMemcpy(p, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes), 1) == 0
        return p.value

    def get(self, ptr: int, like: np.ndarray) -> np.ndarray:
        out = np.empty_like(like)
        assert self.h.hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr),
                                C.c_size_t(out.nbytes), 2) == 0
        return out

    def sync(self):
        assert self.h.hipDeviceSynchronize() == 0

    def free(self):
        for p in self.ptrs:
            self.h.hipFree(p)


def test_device_resident_closed_loop(lqro_mod, oracle, gains):
    """lqro_step_device -> lqro_dynamics_step_device on device buffers, the
    state never leaving HBM: newV feeds vGoal, the new estimate x feeds the
    next pair step (the loop LQRO:1391-1446).  Against the oracle's pair
    step + agent step; 3 control steps."""
    L = lqro_mod.lib()
    n, H, NP = 12, 30, 50
    g = _gains(oracle, l=(0.0, 0.0, 0.0, 0.0))
    x0, vg0 = lqro_mod.synthetic_swarm(n, seed=31, box=3.0)
    st = lqro_mod.agent_states(x0, p_goal=x0[:, :3] + 1.0)
    st["vgoal"][:] = vg0
    ref = {k: v.copy() for k, v in st.items()}
    hip = _Hip()
    try:
        d = {k: hip.put(v) for k, v in st.items()}
        newv_d = hip.put(np.zeros((n, 3)))
        gd = {k: hip.put(np.ascontiguousarray(g[k], np.float64)) for k in ("L", "E", "l", "Lh", "Eh")}
        Md, Nd = hip.put(1e-9 * np.eye(16)), hip.put(1e-9 * np.eye(6))
        models_d = hip.put(np.frombuffer(bytes(lqro_mod.default_model()), dtype=np.uint8))
        ctx = lqro_mod.Context(lqro_mod.config(n, H, NP, flags=0))   # the oracle's default (canonical) rule
        ctx.set_gains(g["A"], g["B"], g["L"], g["E"])
        T, NCF = oracle.tables(g["A"], g["B"], g["L"], g["E"], H)
        S = oracle.sphere(NP)
        seed = 1
        for t in range(3):
            nrm, seed = lqro_mod.normals(seed, n * lqro_mod.NORMALS_PER_AGENT)
            nrm_d = hip.put(nrm)
            assert L.lqro_step_device(ctx._h, C.c_void_p(d["x"]), C.c_void_p(d["vgoal"]),
                                      C.c_void_p(newv_d), None) == 0
            hip.sync()
            assert hip.h.hipMemcpy(C.c_void_p(d["vgoal"]), C.c_void_p(newv_d),
                                   C.c_size_t(n * 3 * 8), 3) == 0          # vGoal = newV
            a = lqro_mod.Agents(*[d[k] for k in STATE], None, d["u_goal"], d["p_goal"],
                                *[gd[k] for k in ("L", "E", "l", "Lh", "Eh")], Md, Nd, nrm_d)
            assert L.lqro_dynamics_step_device(C.c_void_p(models_d), 1, n, 0, C.byref(a), None) == 0
            hip.sync()
            newv_r, _ = oracle.step(T, NCF, S, ref["x"], ref["vgoal"], records=False)
            ref["vgoal"][:] = newv_r
            oracle.agent_step(ref, g, nrm)
            got = {k: hip.get(d[k], ref[k]) for k in STATE}
            _compare(got, ref, 1e-7)
    finally:
        hip.free()


def test_wave_kernel_matches_lane_kernel(lqro_mod, oracle, monkeypatch):
    """k_dynw (one wave per agent, the default) computes every element in the
    same operation order as k_dyn (one lane per agent): bit-identical."""
    n = 96
    g = _gains(oracle)
    st = _states(lqro_mod, n, seed=24)
    other = {k: v.copy() for k, v in st.items()}
    nrm, _ = lqro_mod.normals(5, n * lqro_mod.NORMALS_PER_AGENT)
    monkeypatch.setenv("LQRO_DYN_LANE", "0")
    u0 = lqro_mod.dynamics_step(st, g, nrm)
    monkeypatch.setenv("LQRO_DYN_LANE", "1")
    u1 = lqro_mod.dynamics_step(other, g, nrm)
    assert np.array_equal(u0.view(np.uint64), u1.view(np.uint64))
    for k in STATE:
        assert np.array_equal(st[k].view(np.uint64), other[k].view(np.uint64)), k


def test_simulator_loop(lqro_mod, oracle, tmp_path):
    """The reference-shaped driver: Simulator.step (LQRO:1393-1436) then
    Simulator.update (LQRO:1437-1446), two control steps, against the oracle."""
    n, H, NP = 8, 25, 50
    x0, vg0 = lqro_mod.synthetic_swarm(n, seed=41, box=2.5)
    qs = [lqro_mod.Quadrotor(x0[a], vg0[a], pGoal=-x0[a, :3]) for a in range(n)]
    sim = lqro_mod.Simulator(qs, horizon=H, n_points=NP)
    g = sim.findMatrices()
    g = dict(g, l=np.zeros(4))
    ref = lqro_mod.agent_states(x0, p_goal=-x0[:, :3])
    ref["vgoal"][:] = vg0
    T, NCF = oracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = oracle.sphere(NP)
    seed = seed_ref = 3
    # the Simulator runs the reference's own hull rule (LQRO_FLAG_QHULL_ORDER)
    oracle.set_hull_rule(1, round16=True)
    oracle.carry_normal(np.zeros(3))
    try:
        for t in range(2):
            sim.step()
            seed = sim.update(seed)
            newv, _ = oracle.step(T, NCF, S, ref["x"], ref["vgoal"], records=False)
            ref["vgoal"][:] = newv
            nrm, seed_ref = lqro_mod.normals(seed_ref, n * lqro_mod.NORMALS_PER_AGENT)
            oracle.agent_step(ref, g, nrm)
    finally:
        oracle.set_hull_rule(0)
    got = dict(x=np.stack([q.x for q in qs]), rot=np.stack([q.Rot for q in qs]),
               x_true=np.stack([q.xTrue for q in qs]), rot_true=np.stack([q.RotTrue for q in qs]),
               P=np.stack([q.P for q in qs]), vgoal=np.stack([q.vGoal for q in qs]))
    _compare(got, ref, 1e-7)
    assert seed == seed_ref
    sim.save_trajectory(str(tmp_path / "traj.npz"))
    kf = np.load(tmp_path / "traj.npz")["keyframes"]
    assert kf.shape == (2, n, 8)
    np.testing.assert_array_equal(kf[1, :, 0], np.float32(1 * sim.model.dt))
    np.testing.assert_allclose(kf[1, :, 1:4], got["x_true"][:, :3], rtol=1e-6)
