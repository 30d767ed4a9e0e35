"""k_hull phase profile of one C3 step (needs liblqro_hprof.so, built with
-DLQRO_HULL_PROFILE): per-phase cycles, insertion/conflict counters and the
per-job cycle records."""
import sys, os, ctypes as C, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ.get("LQRO_LIB", "liblqro_hprof.so"))
L = lqro.lib()
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP, flags=0))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
c.step(x, vg)
print(c.timings(), c.stats())
out = np.zeros(32 + 2 * 4096 + 32, np.uint64)
L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
names = {0: "points", 1: "init", 6: "insertions", 8: "final-prep", 9: "final", 15: "job wait"}
tot = sum(int(out[k]) for k in names)
for k, nm in names.items():
    print(f"{nm:14s} {int(out[k]):14d}  {100 * int(out[k]) / max(tot, 1):5.1f}%")
print(f"insertions {int(out[10])}  conflicts (backed off) {int(out[11])}  stale/held pops {int(out[12])}  max region {int(out[13])}  regions > 32: {int(out[14])}  held pops {int(out[32 + 2 * 4096 + 31])}")
print('fail reasons (0=ok):', {k: int(out[16 + k]) for k in range(16) if out[16 + k]})
wn = ["lock", "region", "conflict (wasted)", "horizon+cone", "reassign", "idle", "commit", "wide path", "refill", "held/dead", "apex load"]
wv = out[32 + 2 * 4096 + 16: 32 + 2 * 4096 + 27].astype(float)
print("wave time:", "  ".join(f"{a} {100 * b / max(wv.sum(), 1):.1f}%" for a, b in zip(wn, wv)))
if out[10]:
    print("wave cycles per insertion:", "  ".join(f"{a} {b / out[10]:.0f}" for a, b in zip(wn, wv)))
jobs = out[32:32 + 2 * 4096].reshape(-1, 2)
rows = []
for k, (cyc, w) in enumerate(jobs):
    if cyc == 0:
        continue
    w = int(w)
    rows.append((int(cyc), w & 0xFFFFF, (w >> 20) & 0xFFFFF, (w >> 40) & 0xF, w >> 44, k >= 2048))
rows.sort(reverse=True)
print("jobs:", len(rows), " top by cycles (cycles, vertex slots, n_points, fail, slot, big):")
for r in rows[:12]:
    print("  ", r)
ins = np.array([r[1] for r in rows])
cy = np.array([r[0] for r in rows], float)
print("vertex slots: mean %.0f  max %d;  cycles/job: mean %.0f  max %.0f;  cycles per vertex %.0f"
      % (ins.mean(), ins.max(), cy.mean(), cy.max(), cy.sum() / ins.sum()))
