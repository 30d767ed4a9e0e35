#!/usr/bin/env python3
"""k_dynw phase profile (LQRO_DYN_PROFILE=1, lqro_debug_dyn_profile): the
per-agent step LQRO:1437-1446 for 1024 agents, cycles per phase per agent
(s_memtime), and the step time with and without the stamps."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lqr-obstacles_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "scripts")]
import numpy as np  # noqa: E402

import lqro  # noqa: E402
import pyoracle  # noqa: E402

if os.environ.get("LQRO_LIB"):   # a variant library (its name in lqr-obstacles_amd/)
    lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ["LQRO_LIB"])
from dyn_bench import states  # noqa: E402
from test_gpu_dyn import STATE, _Hip  # noqa: E402

L = lqro.lib()
g = pyoracle.synthesize()
g["l"] = np.array([0.01, -0.02, 0.03, -0.04])
n = 1024
st = states(n, 5)
nrm, _ = lqro.normals(1, n * lqro.NORMALS_PER_AGENT)
hip = _Hip()
d = {k: hip.put(v) for k, v in st.items()}
gd = {k: hip.put(np.ascontiguousarray(g[k], np.float64)) for k in ("L", "E", "l", "Lh", "Eh")}
a = lqro.Agents(*[d[k] for k in STATE], None, d["u_goal"], d["p_goal"], *[gd[k] for k in ("L", "E", "l", "Lh", "Eh")],
                hip.put(1e-9 * np.eye(16)), hip.put(1e-9 * np.eye(6)), hip.put(nrm))
md = hip.put(np.frombuffer(bytes(lqro.default_model()), dtype=np.uint8))
out = np.zeros(32, np.uint64)
L.lqro_debug_dyn_profile.argtypes = [C.c_void_p, C.c_int]
for _ in range(2):
    assert L.lqro_dynamics_step_device(C.c_void_p(md), 1, n, 0, C.byref(a), None) == 0
hip.sync()
L.lqro_debug_dyn_profile(out.ctypes.data_as(C.c_void_p), 1)
reps = 5
t0 = time.perf_counter()
for _ in range(reps):
    assert L.lqro_dynamics_step_device(C.c_void_p(md), 1, n, 0, C.byref(a), None) == 0
hip.sync()
ms = (time.perf_counter() - t0) / reps * 1e3
L.lqro_debug_dyn_profile(out.ctypes.data_as(C.c_void_p), 0)
agents = max(int(out[15]), 1)
names = ["setup+findU", "propagate: discretize", "propagate: noise (jacobi 16)", "kalman1: discretize",
         "kalman1: P update", "observation draw (jacobi 6)", "kalmanFilter2", "findVGoal+store",
         "  discretize: Jacobians", "  discretize: 2 expm", "  discretize: MM, dx"]
tot = sum(int(out[k]) for k in range(8)) + sum(int(out[k]) for k in (8, 9, 10))
print(f"{n} agents, {ms:.3f} ms per step (LQRO_DYN_PROFILE={os.environ.get('LQRO_DYN_PROFILE', '0')}), "
      f"{agents} agent-steps profiled")
for k, nm in enumerate(names):
    v = int(out[k]) / agents
    print(f"  {nm:34s} {v:10.0f} cycles/agent  {100 * int(out[k]) / max(tot, 1):5.1f}%")
print(f"  jacobi<16>: {int(out[11]) / agents:.1f} iterations, {int(out[12]) / agents:.1f} rotations per agent; "
      f"jacobi<6>: {int(out[13]) / agents:.1f} iterations, {int(out[14]) / agents:.1f} rotations")
sub = [("jacobi<16> iteration: scan", 16), ("jacobi<16> iteration: rotation parameters", 17),
       ("jacobi<16> iteration: rotation", 18), ("expm: norm, scale, A2 A4 A6", 19), ("expm: U V, A U, P Q", 20),
       ("expm: solve", 21), ("expm: squarings, copy", 22), ("  solve: elimination", 24),
       ("  solve: back substitution", 25), ("  solve: reshuffle", 26)]
for nm, k in sub:
    print(f"  {nm:44s} {int(out[k]) / agents:10.0f} cycles/agent")
print(f"  expm squarings: {int(out[23]) / agents / 4:.2f} per expm")
