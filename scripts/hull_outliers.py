"""Run many C3 steps and report the hull time distribution; for steps
slower than 1.5x the median, print the slowest jobs (profiling build)."""
import sys, os, ctypes as C, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ.get("LQRO_LIB", "liblqro_hprof.so"))
L = lqro.lib()
N, H, NP = 1024, 100, 100
K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
c.step(x, vg)
prev = np.zeros(32 + 2 * 4096 + 32, np.uint64)
out = np.zeros_like(prev)
L.lqro_debug_hull_profile(c._h, prev.ctypes.data_as(C.c_void_p))
hs = []
for t in range(K):
    c.step(x, vg)
    tm = c.timings()
    L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
    d = out.astype(np.int64) - prev.astype(np.int64)
    hs.append(tm["hull_ms"])
    jobs = out[32:32 + 2 * 4096].reshape(-1, 2)
    cyc = jobs[:, 0].astype(np.int64)
    top = np.argsort(-cyc)[:3]
    print(f"step {t}: hull {tm['hull_ms']:.2f} ms  ins {int(d[10])} conf {int(d[11])} held {int(d[32 + 2 * 4096 + 31])} "
          f"fails { {k: int(d[16 + k]) for k in range(1, 16) if d[16 + k]} } top jobs (Mcyc, vslots): "
          + " ".join(f"({cyc[j] / 1e6:.1f},{int(jobs[j, 1]) & 0xFFFFF})" for j in top), flush=True)
    prev = out.copy()
hs = np.array(hs)
print("hull ms: median %.2f  p90 %.2f  max %.2f" % (np.median(hs), np.percentile(hs, 90), hs.max()))
