"""Time K steps of the C3 swarm (or a denser box) in the default (Qhull-order)
rule through lqro.Context; prints per-step ms and the step's statistics.
usage: c3_step.py [steps] [box side]  (LQRO_LIB: a variant library name)"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro  # noqa: E402

if os.environ.get("LQRO_LIB"):
    lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ["LQRO_LIB"])
K = int(sys.argv[1]) if len(sys.argv) > 1 else 3
box = float(sys.argv[2]) if len(sys.argv) > 2 else None
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N, box=box) if box else lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
for k in range(K):
    t = time.perf_counter()
    c.step(x, vg)
    print(f"step {k}: {1e3 * (time.perf_counter() - t):.2f} ms", c.timings(), c.stats(), flush=True)
