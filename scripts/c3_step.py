"""Time K steps of the C3 swarm (or a denser box) in the default (Qhull-order)
rule through lqro.Context; prints per-step ms and the step's statistics.
usage: c3_step.py [steps] [box side]  (LQRO_LIB: a variant library name; STEP_C4_SHARD=1: BASELINE
config 4's rows [0, 512) of 4096 instead, one rank's work at 8 GPUs)"""
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
shard = {}
if os.environ.get("STEP_C4_SHARD") == "1":
    N, shard = 4096, {"row_begin": 0, "row_end": 512}
x, vg = lqro.synthetic_swarm(N, box=box) if box else lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP, **shard))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
import numpy as np  # noqa: E402

steps = []
for k in range(K):
    t = time.perf_counter()
    c.step(x, vg)
    tm = c.timings()
    b = c.hull_builds()
    dur = (b["t_end"].astype(np.int64) - b["t_start"].astype(np.int64)) / 1e5 if len(b) else np.zeros(1)
    span = (int(b["t_end"].max()) - int(b["t_start"].min())) / 1e5 if len(b) else 0.0
    us_ins = dur.sum() * 1e3 / max(1, int(b["insertions"].sum())) if len(b) else 0.0
    print(f"step {k}: {1e3 * (time.perf_counter() - t):.2f} ms host, {tm['step_ms']:.3f} ms device, "
          f"slowest build {dur.max():.3f} ms, builds span {span:.3f} ms, {us_ins:.2f} us/insertion", c.stats(),
          flush=True)
    if k >= 2:
        steps.append(tm["step_ms"])
if steps:
    print(f"steady: median {np.median(steps):.3f} ms, min {np.min(steps):.3f} ms over {len(steps)} steps", flush=True)
