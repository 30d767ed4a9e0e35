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
out = np.zeros(32, np.uint64)
L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
names = ["points", "init", "select", "visible", "horizon+slots", "cone", "reassign", "retire", "final-prep", "final", "", "", "", "", "iters", "wait"]
tot = out[:14].sum()
for k in range(16):
    if out[k]:
        print(f"{names[k]:14s} {int(out[k]):14d}  {100*out[k]/max(tot,1):5.1f}%")
print('fail reasons (0=ok):', {k: int(out[16+k]) for k in range(16) if out[16+k]})
