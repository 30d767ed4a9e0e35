"""A/B of liblqro variants on the C3 step: argv = variant .so names (in
lqr-obstacles_amd/).  Each variant runs `rounds` x `steps` steps, variants
interleaved; prints median/min/max hull_ms and step_ms."""
import sys, os, importlib, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
names = sys.argv[1:]
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
res = {n: [] for n in names}
base = os.path.dirname(lqro.LIB_PATH)
for rnd in range(3):
    for nm in names:
        importlib.reload(lqro)
        lqro.LIB_PATH = os.path.join(base, nm)
        c = lqro.Context(lqro.config(N, H, NP))
        c.set_gains(g["A"], g["B"], g["L"], g["E"])
        c.step(x, vg)
        for _ in range(4):
            c.step(x, vg)
            res[nm].append(c.timings())
        c.close()
for nm in names:
    h = np.array([t["hull_ms"] for t in res[nm]])
    s = np.array([t["step_ms"] for t in res[nm]])
    p = np.array([t["pair_ms"] for t in res[nm]])
    print(f"{nm:22s} hull med {np.median(h):.2f} min {h.min():.2f} max {h.max():.2f} | pair {np.median(p):.2f} | step med {np.median(s):.2f}", flush=True)
