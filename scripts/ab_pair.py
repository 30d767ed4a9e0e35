"""A/B the pair kernel across builds (interleaved rounds, one process)."""
import sys, os, ctypes as C, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
os.environ.setdefault("LQRO_HOT", "0")   # time k_pair alone
libs = sys.argv[1:]
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
ctxs = []
for path in libs:
    lqro._lib = None
    lqro.LIB_PATH = path
    L = lqro.lib()
    c = lqro.Context(lqro.config(N, H, NP, flags=0))
    c.set_gains(g["A"], g["B"], g["L"], g["E"])
    ctxs.append((path, c, L))
res = {p: [] for p in libs}
for rnd in range(4):
    for path, c, L in ctxs:
        lqro._lib = L
        c.step(x, vg)
        res[path].append(c.timings())
for p in libs:
    t = res[p][1:]
    print(os.path.basename(p), "pair_ms", [round(r["pair_ms"], 2) for r in t], "hull", round(np.median([r["hull_ms"] for r in t]), 2), "lp", round(np.median([r["lp_ms"] for r in t]), 2))
