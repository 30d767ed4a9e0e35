"""The k_qhull caps against the builds of a swarm's inside-hull pairs, on the
CPU oracle (lqro_qhull.c's build statistics): which pairs exceed a cap and
go to k_qhull_big.  usage: qhull_caps.py [box side, default the bench's]"""
import os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), d) for d in ("../oracle", "../lqr-obstacles_amd")]
import lqro, pyoracle as O  # noqa: E402

box = float(sys.argv[1]) if len(sys.argv) > 1 else None
x, vg = lqro.synthetic_swarm(1024, box=box) if box else lqro.synthetic_swarm(1024)
g = O.synthesize()
T, NCF = O.tables(g["A"], g["B"], g["L"], g["E"], 100)
S = O.sphere(100)
_, recs = O.step(T, NCF, S, x, vg, threads=8)
ins = recs[(recs["flags"] & 2) != 0]
print("inside", len(ins))
keys = ["st_horizon_max", "st_cop_max", "st_old_append", "st_visible_max", "st_new_max", "st_partition_max",
        "st_facets_created", "st_addpoints"]
caps = {"st_horizon_max": 24, "st_cop_max": 8, "st_visible_max": 128, "st_new_max": 128}
rows = []
for r in ins:
    i, j = int(r["i"]), int(r["j"])
    _, _, pts = O.pair(T, NCF, S, x[i], x[j], i, j, want_points=True)
    O.qhull(pts)
    st = O.last_qhull_stats
    rows.append([st[k] for k in keys])
    over = [k for k, c in caps.items() if st[k] > c]
    if over:
        print("pair", i, j, "points", len(pts), {k: st[k] for k in keys})
a = np.array(rows)
for k, col in zip(keys, a.T):
    print(f"{k:20s} max {col.max():7d}  p99 {np.percentile(col, 99):9.1f}  mean {col.mean():9.1f}")
