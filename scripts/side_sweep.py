"""C3 step time for several LQRO_HOT / LQRO_SIDE_HULL_CUS settings (one
process; each context reads the environment when it is created)."""
import sys, os, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
settings = [a.split(",") for a in (sys.argv[1:] or ["0,0", "1,64", "1,96", "1,128"])]
ctxs = []
for hot, cus in settings:
    os.environ["LQRO_HOT"] = hot
    os.environ["LQRO_SIDE_HULL_CUS"] = cus
    c = lqro.Context(lqro.config(N, H, NP))
    c.set_gains(g["A"], g["B"], g["L"], g["E"])
    ctxs.append(((hot, cus), c))
res = {k: [] for k, _ in ctxs}
for rnd in range(12):
    for k, c in ctxs:
        c.step(x, vg)
        if rnd == 0:
            print("first step", k, c.timings(), flush=True)
        if rnd >= 2:
            res[k].append(c.timings())
for k, _ in ctxs:
    t = res[k]
    print(f"hot={k[0]} side_cus={k[1]}: step median {np.median([r['step_ms'] for r in t]):.2f} "
          f"max {max(r['step_ms'] for r in t):.2f}  sweep {np.median([r['pair_ms'] for r in t]):.2f} "
          f"hull {np.median([r['hull_ms'] for r in t]):.2f} lp {np.median([r['lp_ms'] for r in t]):.2f}",
          flush=True)
