"""Small hull-branch smoke: the 24-agent parity case and the dense swarm,
GPU vs oracle facet/distance (for debugging the hull kernel)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", d) for d in ("lqr-obstacles_amd", "oracle")]
import numpy as np
import lqro, pyoracle
g = pyoracle.synthesize()
for (N, H, NP, box, seed) in ((24, 50, 100, None, lqro.SEED), (32, 50, 100, 3.0, 11)):
    x, vg = lqro.synthetic_swarm(N, box=box, seed=seed)
    ctx = lqro.Context(lqro.config(N, H, NP, flags=lqro.LQRO_FLAG_RECORDS))
    ctx.set_gains(g["A"], g["B"], g["L"], g["E"])
    ctx.step(x, vg)
    r = ctx.records(); st = ctx.stats(); ctx.close()
    T, NCF = pyoracle.tables(g["A"], g["B"], g["L"], g["E"], H)
    rv, rr = pyoracle.step(T, NCF, pyoracle.sphere(NP), x, vg, threads=8)
    ins = (rr["flags"] & 2) != 0
    same = [np.array_equal(a["facet"], b["facet"]) and a["dist"] == b["dist"] for a, b in zip(r[ins], rr[ins])]
    print(N, st, "inside", int(ins.sum()), "facet+dist exact", sum(same), flush=True)
