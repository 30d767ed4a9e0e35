"""Per-row LP cycles at C3 (liblqro_lpprof.so, -DLQRO_LP_PROFILE)."""
import sys, os, ctypes as C, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), "liblqro_lpprof.so")
L = lqro.lib()
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP, flags=0))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
c.step(x, vg)
print(c.timings())
out = np.zeros(32 + 2 * 4096 + 32, np.uint64)
L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
cy = out[32:32 + N].astype(float)
o = np.argsort(cy)[::-1]
print("LP cycles/row: median %.0f  p99 %.0f  max %.0f" % (np.median(cy), np.percentile(cy, 99), cy.max()))
print("top rows:", [(int(r), int(cy[r])) for r in o[:10]])
info = out[32 + 4096:32 + 4096 + N]
for r in o[:12]:
    v = int(info[r])
    print(f"row {int(r)}: cycles {int(cy[r])}  planes {v >> 40}  lp3 fail at {(v >> 20) & 0xFFFFF}  lp4 iterations {v & 0xFFFFF}")
print("rows in LP4:", int(sum(1 for v in info if (int(v) >> 20) & 0xFFFFF != int(v) >> 40)))
