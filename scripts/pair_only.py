"""Run only the C3 step a few times (for PMC profiling)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
N, H, NP = 1024, 100, 100
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
import os
os.environ.setdefault("LQRO_HOT", "0")   # one k_pair launch over all pairs
ctx = lqro.Context(lqro.config(N, H, NP, flags=0))
ctx.set_gains(g["A"], g["B"], g["L"], g["E"])
for _ in range(steps):
    ctx.step(x, vg)
print(ctx.stats(), ctx.timings())
