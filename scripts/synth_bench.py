"""Batched gain synthesis: C5's 16384 heterogeneous
agents on the GPU (lqro_synthesize_gains_batch_x; k_synthw one wave per
agent, and the one-lane k_synth with LQRO_SYNTH_LANE=1) vs the host path of
the same source on one core, for X = 16 and 12.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
models = lqro.perturbed_models(n)
out = {"what": "controlMatrices x N heterogeneous agents (LQRO:520-582)", "agents": n}
for X in (16, 12):
    for kern, env in (("k_synthw", "0"), ("k_synth", "1")):
        os.environ["LQRO_SYNTH_LANE"] = env
        lqro.synthesize_gains_batch(models[:64], x_dim=X)     # first launch: code object, scratch
        ts = []
        for _ in range(2):
            t0 = time.perf_counter()
            g = lqro.synthesize_gains_batch(models, x_dim=X)
            ts.append(time.perf_counter() - t0)
        k = 8
        t0 = time.perf_counter()
        host = [lqro.synthesize_gains(m, x_dim=X) for m in models[:k]]
        t_host = (time.perf_counter() - t0) / k
        ok = all(np.array_equal(g[key][j], host[j][key]) for j in range(k) for key in host[0])
        out[f"x{X}_{kern}"] = {"gpu_s": min(ts), "agents_per_s": n / min(ts), "host_s_per_agent_1core": t_host,
                               "gpu_over_1core": t_host * n / min(ts), "bit_exact_vs_host_first8": ok}
print(json.dumps(out), flush=True)
