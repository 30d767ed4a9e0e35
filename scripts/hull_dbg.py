"""Hull failure diagnosis: one step with the -DLQRO_HULL_PROFILE build,
prints fail-reason counts and per-job records.  argv: N H NP [seed] [box]"""
import sys, os, ctypes as C, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), "liblqro_hprof.so")
L = lqro.lib()
N, H, NP = (int(a) for a in sys.argv[1:4])
seed = int(sys.argv[4]) if len(sys.argv) > 4 else None
box = float(sys.argv[5]) if len(sys.argv) > 5 else None
kw = {}
if seed is not None: kw["seed"] = seed
if box is not None: kw["box"] = box
x, vg = lqro.synthetic_swarm(N, **kw)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
c.step(x, vg)
print(c.timings(), c.stats())
out = np.zeros(32 + 2 * 4096 + 32, np.uint64)
L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
print(f"insertions {int(out[10])}  conflicts {int(out[11])}  stale {int(out[12])}")
print('fail reasons (0=ok):', {k: int(out[16 + k]) for k in range(16) if out[16 + k]})
jobs = out[32:32 + 2 * 4096].reshape(-1, 2)
for k, (cyc, w) in enumerate(jobs):
    if cyc:
        w = int(w)
        print("job", k, "cycles", int(cyc), "vslots", w & 0xFFFFF, "n", (w >> 20) & 0xFFFFF, "fail", (w >> 40) & 0xF, "slot", w >> 44)
