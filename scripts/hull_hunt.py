"""Run the C3 step many times with the production library and report every
step whose hull phase is slow, with the hull outcome codes of that step
(prof[16 + code]: 0 ok, 1-4 and 11 LDS-capacity retries, ...)."""
import sys, os, ctypes as C, numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro
L = lqro.lib()
N, H, NP = 1024, 100, 100
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
prev = np.zeros(32 + 2 * 4096 + 32, np.uint64)
hs = []
for t in range(steps):
    c.step(x, vg)
    out = np.zeros_like(prev)
    L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
    d = out - prev
    prev = out
    tm = c.timings()
    hs.append(tm["hull_ms"])
    codes = {k: int(d[16 + k]) for k in range(16) if d[16 + k]}
    if tm["hull_ms"] > 8 or set(codes) - {0}:
        print(f"step {t}: pair {tm['pair_ms']:.2f} hull {tm['hull_ms']:.2f} codes {codes}", flush=True)
hs = np.array(hs)
print(f"hull ms: median {np.median(hs):.2f} p90 {np.percentile(hs, 90):.2f} max {hs.max():.2f}")
