"""C3 step time vs k_prio's hot radius / horizon (env LQRO_HOT_R / LQRO_HOT_T),
one context per setting, created and used in turn."""
import sys, os, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
for spec in sys.argv[1:]:
    r, t, cus = spec.split(",")
    os.environ["LQRO_HOT_R"], os.environ["LQRO_HOT_T"], os.environ["LQRO_SIDE_HULL_CUS"] = r, t, cus
    c = lqro.Context(lqro.config(N, H, NP))
    c.set_gains(g["A"], g["B"], g["L"], g["E"])
    ts = []
    for k in range(8):
        c.step(x, vg)
        if k >= 2:
            ts.append(c.timings())
    print(f"r={r} t={t} side={cus}: step {np.median([q['step_ms'] for q in ts]):.2f} "
          f"sweep {np.median([q['pair_ms'] for q in ts]):.2f} post-hull {np.median([q['hull_ms'] for q in ts]):.3f}",
          flush=True)
    c.close()
