#!/usr/bin/env python3
"""Golden fixture: the C3 swarm's hardest new-velocity LPs (calculateNewV,
LQRO:1223-1234 — linearProgram3 fails, linearProgram4 runs).

TEST INFRASTRUCTURE, build container.  One oracle step of C3 (1,024
agents, H 100, NP 100, Qhull order, tests/golden/qhull_order.npz pins that
step to live Qhull) gives every row's 1,023 ORCA planes in push order; the
rows whose LP reaches linearProgram4 are ranked by the length of their
sequential chain (linearProgram1 calls + violated-plane scans), and the
slowest ones are kept with their goals and the oracle's new velocities.
Writes tests/golden/lp_rows.npz (planes float32 [R, 1023, 6], vgoal
[R, 3], newv [R, 3], rows [R], vmax_lp).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "lqr-obstacles_amd")]
import pyoracle  # noqa: E402
import lqro  # noqa: E402

KEEP = 8


def main():
    pyoracle.lib()
    N, H, NP = 1024, 100, 100
    x, vg = lqro.synthetic_swarm(N)
    g = pyoracle.synthesize()
    T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    S = pyoracle.sphere(NP)
    pyoracle.set_hull_rule(1, round16=False)
    pyoracle.carry_normal(np.zeros(3))
    v, r = pyoracle.step(T, NCF, S, x, vg, threads=8)
    pyoracle.set_hull_rule(0)
    R = r.reshape(N, N - 1)
    assert ((R["flags"] & lqro.REC_PLANE) != 0).all()
    pl = np.concatenate([R["plane_point"], R["plane_normal"]], 2).astype(np.float32)
    vmax = float(lqro.config(N, H, NP).vmax_lp)
    cost = np.array([pyoracle.lp_chain(pl[i], vg[i], vmax) for i in range(N)])
    rows = np.argsort(-cost)[:KEEP]
    rows = rows[cost[rows] > 0]
    nv = np.array([pyoracle.newv(pl[i], vg[i], vmax) for i in rows])
    assert np.array_equal(nv, v[rows])
    # pinned to the reference's own calculateNewV (oracle/_ref, maxSpeed_ 100)
    r = pyoracle.reflib()
    if r is not None and vmax == 100.0:
        import ctypes as C
        for k, i in enumerate(rows):
            p6 = np.ascontiguousarray(pl[i])
            out = np.zeros(3)
            gv = np.ascontiguousarray(vg[i], np.float64)
            r.ref_newv(p6.shape[0], p6.ctypes.data_as(C.c_void_p), gv.ctypes.data_as(C.c_void_p),
                       out.ctypes.data_as(C.c_void_p))
            assert np.array_equal(out, nv[k]), i
        print("pinned to ref_newv")
    np.savez_compressed(os.path.join(HERE, "lp_rows.npz"), planes=pl[rows], vgoal=vg[rows], newv=nv,
                        rows=rows, vmax_lp=vmax, chain=cost[rows])
    print("rows", rows.tolist(), "chain", cost[rows].tolist())


if __name__ == "__main__":
    main()
