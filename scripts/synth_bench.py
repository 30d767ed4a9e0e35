"""Batched gain synthesis: C5's 16384 heterogeneous
agents on the GPU (lqro_synthesize_gains_batch) vs the host path of the same
source, one core.  Prints one JSON line."""
import json, os, sys, time
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
rng = np.random.default_rng(1)
models = []
for _ in range(n):
    m = lqro.default_model()
    for f in ("mass", "inertia", "thrust_latency", "length", "qv", "qp", "r"):
        setattr(m, f, getattr(m, f) * (1.0 + rng.uniform(-0.01, 0.01)))
    models.append(m)
t0 = time.perf_counter()
lqro.synthesize_gains_batch(models[:64])            # first launch: code object, scratch
t_first = time.perf_counter() - t0
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    out = lqro.synthesize_gains_batch(models)
    ts.append(time.perf_counter() - t0)
t_gpu = min(ts)
k = 16
t0 = time.perf_counter()
host = [lqro.synthesize_gains(m) for m in models[:k]]
t_host = (time.perf_counter() - t0) / k
ok = all(np.array_equal(out[key][j], host[j][key]) for j in range(k) for key in lqro.GAIN_SHAPES)
print(json.dumps({"what": "controlMatrices x N heterogeneous agents (LQRO:520-582)", "agents": n,
                  "gpu_s": t_gpu, "gpu_s_runs": ts, "gpu_first_launch_s": t_first,
                  "gpu_agents_per_s": n / t_gpu, "host_s_per_agent_1core": t_host,
                  "host_agents_per_s_1core": 1.0 / t_host, "gpu_over_1core": t_host * n / t_gpu,
                  "bit_exact_vs_host_first16": ok}), flush=True)
