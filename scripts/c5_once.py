"""One GPU shard of BASELINE config 5 (16384 agents, X = 12 reduced model,
per-agent +-1 % gains, H = 200, rows [0, 2048)), a few steps; prints the
step timings and stats (for rocprofv3 kernel traces).  LQRO_HOT selects the
schedule as in liblqro."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd"))
import lqro  # noqa: E402

N, H, NP, X = 16384, 200, 100, 12
rows = (0, int(os.environ.get("C5_ROWS", "2048")))
steps = int(os.environ.get("C5_STEPS", "2"))
g = lqro.synthesize_gains_batch(lqro.perturbed_models(N), x_dim=X)
A, B = lqro.synthesize_gains(x_dim=X)["A"], lqro.synthesize_gains(x_dim=X)["B"]
x, vg = lqro.synthetic_swarm(N, x_dim=X)
ctx = lqro.Context(lqro.config(N, H, NP, x_dim=X, row_begin=rows[0], row_end=rows[1], flags=0))
ctx.set_gains(A, B, g["L"], g["E"], per_agent=True)
for s in range(steps):
    t0 = time.perf_counter()
    ctx.step(x, vg)
    print(f"step {s}: {(time.perf_counter() - t0) * 1e3:.1f} ms", ctx.timings(), ctx.stats(), flush=True)
ctx.close()

# hull outcome histogram (liblqro's always-on counters: code 0 = ok, 1 = vertex
# capacity, 4 = face capacity, 6 = segment buffer, 9 = stall guard, 11 = queue)
import ctypes as C  # noqa: E402
import numpy as np  # noqa: E402
ctx = lqro.Context(lqro.config(N, H, NP, x_dim=X, row_begin=rows[0], row_end=rows[1], flags=0))
ctx.set_gains(A, B, g["L"], g["E"], per_agent=True)
ctx.step(x, vg)
out = np.zeros(32 + 2 * 4096 + 32, np.uint64)
lqro.lib().lqro_debug_hull_profile(ctx._h, out.ctypes.data_as(C.c_void_p))
print("hull outcomes (code: count):", {k: int(out[16 + k]) for k in range(16) if out[16 + k]})
jobs = out[32:32 + 2 * 2048].reshape(-1, 2)
nv = jobs[:, 1] & 0xFFFFF
npts = (jobs[:, 1] >> 20) & 0xFFFFF
ok = jobs[:, 0] > 0
print("jobs recorded", int(ok.sum()), "vertices p50/p90/max", np.percentile(nv[ok], [50, 90, 100]) if ok.any() else None,
      "points p50/max", np.percentile(npts[ok], [50, 100]) if ok.any() else None)
ctx.close()
