"""BASELINE config 5's whole swarm (16384 agents, X = 12, H = 200, per-agent
gains) on one GPU in Qhull order through step_rows, a few steps: per step the
host time, the context's timings and counters, the builds (count, slowest,
total CU time) — for the schedule's A/B (LQRO_* knobs in the environment).
usage: c5_whole.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd"))
import lqro  # noqa: E402
import numpy as np  # noqa: E402

N, H, NP, X = 16384, 200, 100, 12
K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
g = lqro.synthesize_gains_batch(lqro.perturbed_models(N), x_dim=X)
A, B = lqro.synthesize_gains(x_dim=X)["A"], lqro.synthesize_gains(x_dim=X)["B"]
x, vg = lqro.synthetic_swarm(N, x_dim=X)
ctx = lqro.Context(lqro.config(N, H, NP, x_dim=X))
ctx.set_gains(A, B, g["L"], g["E"], per_agent=True)
tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("LQRO_")) or "defaults"
for s in range(K):
    t0 = time.perf_counter()
    try:
        ctx.step(x, vg)
    except lqro.QhullMergeSuspect:
        pass
    ms = (time.perf_counter() - t0) * 1e3
    b = ctx.hull_builds()
    d = (b["t_end"] - b["t_start"]) / 1e5
    st = ctx.stats()
    print(f"[{tag}] step {s}: {ms:.1f} ms {ctx.timings()} inside {st['inside']} retried {st['qhull_retried']}; "
          f"builds {len(b)} slowest {d.max():.1f} ms, sum {d.sum():.0f} CU-ms", flush=True)
ctx.close()
