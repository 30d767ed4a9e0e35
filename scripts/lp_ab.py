"""LP time (k_lp_lds + k_lp4) at C3 across builds: argv = library paths."""
import sys, os, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
for path in sys.argv[1:]:
    lqro._lib = None
    lqro.LIB_PATH = path
    c = lqro.Context(lqro.config(N, H, NP))
    c.set_gains(g["A"], g["B"], g["L"], g["E"])
    t = []
    for k in range(6):
        c.step(x, vg)
        if k:
            t.append(c.timings())
    print(os.path.basename(path), "lp", [round(r["lp_ms"], 3) for r in t], "step", round(np.median([r["step_ms"] for r in t]), 2), flush=True)
    c.close()
