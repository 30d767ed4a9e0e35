"""One 8-way shard of BASELINE config 5 (16384 agents, X = 12, per-agent
+-1 % gains, H = 200) in Qhull order (the default), a few steps through
lqro_step: per step the host time, the context's HIP-event timings (sweep,
hulls, LP) and counters.  C5_SHARD (0..7, default 3), C5_STEPS (default 3).
For rocprofv3 kernel traces of one shard."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd"))
import lqro  # noqa: E402
import numpy as np  # noqa: E402

N, H, NP, X = 16384, 200, 100, 12
g8 = int(os.environ.get("C5_SHARD", "3"))
rows = (g8 * N // 8, (g8 + 1) * N // 8)
steps = int(os.environ.get("C5_STEPS", "3"))
g = lqro.synthesize_gains_batch(lqro.perturbed_models(N), x_dim=X)
A, B = lqro.synthesize_gains(x_dim=X)["A"], lqro.synthesize_gains(x_dim=X)["B"]
x, vg = lqro.synthetic_swarm(N, x_dim=X)
ctx = lqro.Context(lqro.config(N, H, NP, x_dim=X, row_begin=rows[0], row_end=rows[1]))
ctx.set_gains(A, B, g["L"], g["E"], per_agent=True)
for s in range(steps):
    t0 = time.perf_counter()
    try:
        ctx.step(x, vg)
    except lqro.QhullMergeSuspect:
        pass
    print(f"shard {g8} rows {rows} step {s}: {(time.perf_counter() - t0) * 1e3:.1f} ms", ctx.timings(), ctx.stats(),
          flush=True)
b = ctx.hull_builds()
if len(b):
    d = (b["t_end"] - b["t_start"]) / 1e5
    print(f"builds {len(b)}: slowest {d.max():.2f} ms, mean {d.mean():.2f} ms, kernels {sorted(set(b['kernel'].tolist()))}")
    if os.environ.get("C5_TIMELINE"):
        t0 = b["t_start"].min()
        o = np.argsort(b["t_start"])
        print("builds by start (ms from the first): start end dur kernel points insertions")
        for k in o:
            print(f"{(b['t_start'][k] - t0) / 1e5:9.2f} {(b['t_end'][k] - t0) / 1e5:9.2f} {d[k]:8.2f} {b['kernel'][k]} "
                  f"{b['n_points'][k]} {b['insertions'][k]}")
ctx.close()
