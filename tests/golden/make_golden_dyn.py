#!/usr/bin/env python3
"""Generate tests/golden/dyn.npz from the REFERENCE's own code.

TEST INFRASTRUCTURE.  Runs only in the build container (needs
oracle/_ref/libref.so, built from /root/reference by oracle/Makefile).  Stores
inputs and the reference's outputs of the per-agent step after the pair loop:

  l                     controlMatrices' l (LQRO:552,557) at hover
  ctl_*                 riccatiControllerSteady (LQRO:594-617) and
                        riccatiControllerSteadyPosition (LQRO:619-645)
  k1_*                  kalmanFilter1 (LQRO:488-505)
  k2_*                  kalmanFilter2 (LQRO:507-518)
  quat_*                quatFromRot (stdafx.h:24-33), Quadrotor::visualize's
                        keyframe orientation (LQRO:128-133)

propagate (LQRO:473-486) and the observation draw call sampleGaussian, whose
jacobi needs MSVC's _hypot (not in this image): they have no fixture; the
tests pin them through kalmanFilter1 and jacobi's properties.

Usage:  python tests/golden/make_golden_dyn.py
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import pyoracle  # noqa: E402
from dyn_cases import quat_cases, random_agent_cases  # noqa: E402


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def main():
    r = pyoracle.reflib()
    if r is None:
        raise SystemExit("needs oracle/_ref/libref.so (/root/reference)")
    g = pyoracle.synthesize()
    l = np.zeros(4)
    r.ref_gain_l(_p(l))
    cs = random_agent_cases(24, seed=0x44594E)
    n = cs["x"].shape[0]
    u = np.zeros((n, 4))
    v = np.zeros((n, 3))
    k1 = {k: cs[k].copy() for k in ("x", "rot", "P")}
    k2 = {k: cs[k].copy() for k in ("x", "rot", "P")}
    for a in range(n):
        r.ref_control_velocity(_p(cs["x"][a]), _p(cs["rot"][a]), _p(cs["vgoal"][a]),
                               _p(cs["u_goal"][a]), _p(g["L"]), _p(g["E"]), _p(l), _p(u[a]))
        r.ref_control_position(_p(cs["x"][a]), _p(cs["rot"][a]), _p(cs["p_goal"][a]),
                               _p(cs["u_goal"][a]), _p(g["Lh"]), _p(g["Eh"]), _p(v[a]))
        r.ref_kalman1(_p(k1["x"][a]), _p(k1["rot"][a]), _p(u[a]), _p(k1["P"][a]))
        r.ref_kalman2(_p(k2["x"][a]), _p(k2["rot"][a]), _p(cs["z"][a]), _p(k2["P"][a]))
    qin = quat_cases()
    qout = np.zeros((qin.shape[0], 4))
    for a in range(qin.shape[0]):
        r.ref_quat_from_rot(_p(qin[a]), _p(qout[a]))
    out = dict(l=l, u=u, v=v, quat_in=qin, quat_out=qout, **{"in_" + k: val for k, val in cs.items()},
               **{"k1_" + k: val for k, val in k1.items()},
               **{"k2_" + k: val for k, val in k2.items()})
    np.savez_compressed(os.path.join(HERE, "dyn.npz"), **out)
    print("wrote dyn.npz:", {k: val.shape for k, val in out.items()})


if __name__ == "__main__":
    main()
