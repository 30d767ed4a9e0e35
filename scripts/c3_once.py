"""One C3 step with timings (smoke of the full pipeline)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
if len(sys.argv) > 1:
    lqro.LIB_PATH = sys.argv[1]
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
for k in range(3):
    c.step(x, vg)
    print(c.timings(), flush=True)
