"""Hull failures in Qhull order on a C5 shard (rows [0, 2048) of 16,384
agents, X = 12, H = 200, per-agent gains): each failed pair's status bits
(record n_facets = -(status) - 1) and point count."""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro  # noqa: E402

N, H, NP, X = 16384, 200, 100, 12
chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
x, vg = lqro.synthetic_swarm(N, x_dim=X)
g = lqro.synthesize_gains_batch(lqro.perturbed_models(N), x_dim=X)
g0 = lqro.synthesize_gains(x_dim=X)
for rb in range(0, N, chunk):
    re = min(N, rb + chunk)
    c = lqro.Context(lqro.config(N, H, NP, x_dim=X, row_begin=rb, row_end=re,
                                 flags=lqro.LQRO_FLAG_RECORDS | lqro.LQRO_FLAG_QHULL_ORDER))
    c.set_gains(g0["A"], g0["B"], g["L"], g["E"], per_agent=True)
    c.step(x, vg)
    st = c.stats()
    r = c.records()
    bad = r[(r["flags"] & lqro.REC_HULLFAIL) != 0]
    print(rb, re, st, flush=True)
    for b in bad:
        print("  pair", int(b["i"]), int(b["j"]), "n_reach", int(b["n_reach"]), "status", -int(b["n_facets"]) - 1,
              flush=True)
    del r
    c.close()
