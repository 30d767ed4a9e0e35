import sys, os, ctypes as C, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), "liblqro_hprof.so")
L = lqro.lib()
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
c.step(x, vg)
print(c.timings(), c.stats())
out = np.zeros(32 + 2 * 4096 + 16, np.uint64)
L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
names = ["points", "init", "candidates", "regions", "accept", "cone", "reassign", "retire", "final-prep", "final", "candidates", "rounds", "sum moved", "", "insertions", "wait"]
tot = out[:10].sum()
for k in range(16):
    if out[k]:
        pct = f"{100*out[k]/max(tot,1):5.1f}%" if k < 10 else ""
        print(f"{names[k]:14s} {int(out[k]):14d}  {pct}")
print('fail reasons (0=ok):', {k: int(out[16+k]) for k in range(13) if out[16+k]})
print('reassign sub-phases (pre, load q, tests, ballots, stores, seg):', [int(v) for v in out[26:32]])

jobs = out[32:].reshape(-1, 2)
rows = []
for k, (cyc, w) in enumerate(jobs):
    if cyc == 0:
        continue
    w = int(w)
    rows.append((int(cyc), w & 0xFFFFF, (w >> 20) & 0xFFFFF, (w >> 40) & 0xF, w >> 44, k >= 2048))
rows.sort(reverse=True)
print("jobs:", len(rows), " top by cycles (cycles, vertices/insertions, n_points, fail, slot, big):")
for r in rows[:12]:
    print("  ", r)
ins = np.array([r[1] for r in rows])
print("insertions: mean %.0f  p50 %.0f  p90 %.0f  max %d" % (ins.mean(), np.median(ins), np.percentile(ins, 90), ins.max()))
cy = np.array([r[0] for r in rows], float)
print("cycles/insertion: mean %.0f" % (cy.sum() / ins.sum()))
