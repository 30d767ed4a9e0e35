"""Estimate multi-GPU step time on one GPU: run each rank's row shard of the
headline step (lqro.shard_rows, block and cyclic) in turn and report per-rank
device time; the max is what N GPUs would take (plus the all-gather).  The
swarm grows as bench.py's weak scaling does: N = round(1024 sqrt(world)).
argv: worlds (default 1,2,4,8), scenario: uniform (bench.py's swarm) or
clustered (the first N/8 agents packed into a box 1/8 the size)."""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import numpy as np
import lqro

H, NP = 100, 100
g = lqro.synthesize_gains()
worlds = [int(w) for w in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("1", "2", "4", "8"))]
scenario = sys.argv[2] if len(sys.argv) > 2 else "uniform"
out = []
for world in worlds:
    N = int(round(1024 * world ** 0.5))
    x, vg = lqro.synthetic_swarm(N)
    if scenario == "clustered":
        # a formation at the front of the index space: the first N/8 agents in
        # a box 1/8 the size, so their rows carry most of the inside-hull pairs
        k = N // 8
        x[:k, 0:3] *= 0.125
    for mode in ("block", "cyclic"):
        times = []
        for r in range(world):
            c = lqro.Context(lqro.config(N, H, NP, **lqro.shard_rows(N, r, world, mode)))
            c.set_gains(g["A"], g["B"], g["L"], g["E"])
            c.step(x, vg)
            ts = []
            for _ in range(3):
                c.step(x, vg)
                ts.append(c.timings())
            st = c.stats()
            c.close()
            times.append(dict(step=float(np.median([t["step_ms"] for t in ts])),
                              pair=float(np.median([t["pair_ms"] for t in ts])),
                              hull=float(np.median([t["hull_ms"] for t in ts])), inside=int(st["inside"])))
        worst = max(t["step"] for t in times)
        mean = float(np.mean([t["step"] for t in times]))
        rec = dict(world=world, n_agents=N, scenario=scenario, mode=mode, max_step_ms=worst, mean_step_ms=mean,
                   imbalance=worst / mean, ranks=times)
        out.append(rec)
        print(f"world {world} N {N} {mode:6s}: max {worst:.2f} ms mean {mean:.2f} imbalance {worst / mean:.3f} ",
              " ".join(f"[{t['step']:.1f} h{t['hull']:.1f} i{t['inside']}]" for t in times), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
with open(f"gpurun_out/rank_sim_{scenario}.json", "w") as f:
    json.dump(out, f, indent=1)
