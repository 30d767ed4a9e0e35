"""Estimate multi-GPU step time on one GPU: run each rank's row shard of the
C3 step (lqro.row_shard) in turn and report per-rank device time; the max is
what N GPUs would take (plus the all-gather)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import numpy as np
import lqro
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
for world in (1, 2, 4, 8):
    times = []
    for r in range(world):
        rb, re = lqro.row_shard(N, r, world)
        c = lqro.Context(lqro.config(N, H, NP, row_begin=rb, row_end=re))
        c.set_gains(g["A"], g["B"], g["L"], g["E"])
        c.step(x, vg)
        ts = []
        for _ in range(3):
            c.step(x, vg)
            ts.append(c.timings())
        st = c.stats()
        c.close()
        times.append((np.median([t["step_ms"] for t in ts]), np.median([t["pair_ms"] for t in ts]),
                      np.median([t["hull_ms"] for t in ts]), st["inside"]))
    worst = max(t[0] for t in times)
    print(f"world {world}: max step {worst:.2f} ms  speedup {times[0][0] if world == 1 else 0:.2f}",
          " ".join(f"[{t[0]:.1f} p{t[1]:.1f} h{t[2]:.1f} i{t[3]}]" for t in times), flush=True)
