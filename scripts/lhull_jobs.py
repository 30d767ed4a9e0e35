"""Per-job profile of k_lhull (the local hull, lqro_lhull.hpp) on one swarm:
point generation and hull-loop wall time (s_memrealtime, 100 MHz), loop
iterations, local vertices / faces, live points after compaction.
usage: lhull_jobs.py [box]   (default: the C3 bench swarm)"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lqr-obstacles_amd")]
os.environ.setdefault("LQRO_LOCAL_HULL", "1")
os.environ.setdefault("LQRO_LHULL_PROFILE", "1")   # k_lhull writes its per-job words
import lqro  # noqa: E402

box = float(sys.argv[1]) if len(sys.argv) > 1 else None
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N, box=box, seed=7) if box else lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
ctx = lqro.Context(lqro.config(N, H, NP, flags=0))
ctx.set_gains(g["A"], g["B"], g["L"], g["E"])
for _ in range(3):
    ctx.step(x, vg)
t = ctx.timings()
buf = (C.c_ulonglong * (4 * 4096))()
lqro.lib().lqro_debug_local_hull_jobs.argtypes = [C.c_void_p, C.c_void_p]
assert lqro.lib().lqro_debug_local_hull_jobs(ctx._h, buf) == 0
st = ctx.stats()
ctx.close()
J = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4)[: min(st["inside"], 4096)]
pts_us = (J[:, 0] & 0xFFFFFFFF) / 100.0
set_us = (J[:, 0] >> 32) / 100.0
loop_us = (J[:, 1] & 0xFFFFFFFF) / 100.0
comp_us = (J[:, 1] >> 32) / 100.0
ncomp = J[:, 3] >> 56
it = J[:, 2] & 0xFFFF
nv = (J[:, 2] >> 16) & 0xFFFF
nc = (J[:, 2] >> 32) & 0xFFFF
grid = J[:, 2] >> 48
blk = (J[:, 3] >> 16) & 0xFFFF
n = J[:, 3] & 0xFFFF
fail = (J[:, 3] >> 32) & 0xFF
nf = (J[:, 3] >> 40) & 0xFFFF
print(f"inside pairs {st['inside']}, timings {t}")
for name, v in (("points us", pts_us), ("hull us", loop_us), ("  setup us", set_us), ("  compact us", comp_us),
                ("  compactions", ncomp), ("iterations", it), ("vertices", nv),
                ("faces (slots)", nf), ("live points", nc), ("points", n)):
    print(f"  {name:14s} mean {v.mean():9.1f}  median {np.median(v):9.1f}  max {v.max():9.1f}")
it_us = (loop_us - set_us - comp_us) / np.maximum(it, 1)
print(f"  us / iteration (excl. setup, compaction): mean {it_us.mean():.2f}; handed over {int((fail != 0).sum())}")
for g in sorted(set(grid.tolist())):
    sel = grid == g
    tot = pts_us[sel] + loop_us[sel]
    print(f"  launch of {g} workgroups: {int(sel.sum())} jobs (queue positions {np.flatnonzero(sel).min()}..{np.flatnonzero(sel).max()}), "
          f"points+hull us mean {tot.mean():.0f} max {tot.max():.0f}")
