"""The C3 step's Qhull-order builds under the current schedule (env: any
LQRO_* knob): per step the step time, the slowest build and its us per
insertion, the mean build — to see whether the builds run slower beside the
sweep (clock / memory contention) than alone (LQRO_HOT=0: the sweep first,
then the builds on an idle chip).  usage: c3_builds.py [steps]"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro  # noqa: E402
import numpy as np  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
N, H, NP = 1024, 100, 100
if os.environ.get("STEP_C4_SHARD") == "1":
    N = 4096
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
shard = {"row_begin": 0, "row_end": 512} if N == 4096 else {}
c = lqro.Context(lqro.config(N, H, NP, **shard))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("LQRO_")) or "defaults"
for k in range(K):
    t = time.perf_counter()
    c.step(x, vg)
    ms = (time.perf_counter() - t) * 1e3
    tm = c.timings()
    b = c.hull_builds()
    b = b[b["kernel"] != 2]
    d = (b["t_end"] - b["t_start"]) / 1e5
    w = int(np.argmax(d))
    span = (b["t_end"].max() - b["t_start"].min()) / 1e5
    print(f"[{tag}] step {k}: host {ms:.2f} ms device {tm['step_ms']:.2f} ms; builds {len(b)} span {span:.2f} ms, "
          f"slowest {d[w]:.3f} ms ({b['insertions'][w]} ins, {1e3 * d[w] / b['insertions'][w]:.2f} us/ins), "
          f"mean {d.mean():.3f} ms, {1e3 * d.sum() / b['insertions'].sum():.2f} us/ins", flush=True)
c.close()
