"""Time K steps of BASELINE config 4 (4096 quadrotors, H 100, one GPU, the
default Qhull-order step) through lqro.Context; prints per-step ms, the
step's event timings and statistics.  usage: c4_step.py [steps]"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 3
N, H, NP = 4096, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
for k in range(K):
    t = time.perf_counter()
    c.step(x, vg)
    print(f"step {k}: {1e3 * (time.perf_counter() - t):.2f} ms", c.timings(), c.stats(), flush=True)
