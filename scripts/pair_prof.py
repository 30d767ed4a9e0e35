"""Per-phase cycle profile of k_pair at C3 (liblqro_pprof.so, -DLQRO_PAIR_PROFILE)."""
import sys, os, ctypes as C, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), "liblqro_pprof.so")
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
pp = out[32 + 2 * 4096:]
names = ["tables->LDS", "classify", "mixed", "", "gjk", "write", "", "loop-top"]
tot = pp[:8].sum() - pp[3] - pp[6]   # [3], [6]: inside gjk (support eval, johnson)
for k in range(8):
    if pp[k] and names[k]:
        print(f"{names[k]:12s} {int(pp[k]):14d} {100 * pp[k] / tot:5.1f}%")
pairs = int(pp[11])
print("pairs", pairs, "mixed slices/pair %.2f" % (pp[10] / max(pairs, 1)),
      "supports/pair %.2f" % (pp[13] / max(pairs, 1)),
      "support cycles/pair %.0f (%.1f%% of gjk)" % (pp[12] / max(pairs, 1), 100 * pp[12] / max(pp[4], 1)),
      "candidates/support %.2f" % (pp[14] / max(pp[13], 1)),
      "cycles/pair/wave %.0f" % (tot / max(pairs, 1)))
print("gjk cycles/pair: johnson %.0f witness %.0f support %.0f (bounds+argmax %.0f, first slice %.0f) point %.0f" %
      tuple(v / max(pairs, 1) for v in (pp[6], pp[8], pp[12], pp[15], pp[3], pp[9])))
