#!/usr/bin/env python3
"""Step time with opt-in neighbour culling (lqro_set_neighbors) at swarm sizes
where all-pairs is out of reach for one GPU: N agents at C3's density
(box 4 N^(1/3) m), H = 100, NP = 100, each agent keeping its k nearest within
r metres.  Writes gpurun_out/nbr_bench.json."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lqr-obstacles_amd"))
import lqro  # noqa: E402


def main():
    g = lqro.synthesize_gains()
    out = []
    for N, k, r in ((4096, 16, 6.0), (16384, 16, 6.0), (16384, 32, 8.0)):
        x, vg = lqro.synthetic_swarm(N)
        ctx = lqro.Context(lqro.config(N, 100, 100, flags=0))
        ctx.set_gains(g["A"], g["B"], g["L"], g["E"])
        ctx.set_neighbors(r, k)
        ctx.step(x, vg)
        reps = 5
        t0 = time.perf_counter()
        dev = 0.0
        for _ in range(reps):
            ctx.step(x, vg)
            dev += ctx.timings()["step_ms"]
        wall = (time.perf_counter() - t0) / reps * 1e3
        st = ctx.stats()
        row = {"agents": N, "max_neighbors": k, "neighbor_dist_m": r, "pairs_kept": st["pairs"],
               "inside_hull": st["inside"], "step_ms_device": dev / reps, "step_ms_wall_host_arrays": wall,
               "kept_pair_evals_per_s": st["pairs"] / (dev / reps) * 1e3}
        print(json.dumps(row), flush=True)
        out.append(row)
        del ctx
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "nbr_bench.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
