"""Repeat one step many times (the concurrent hull is scheduled differently
each run) and check every inside-hull record against the oracle.
argv: N H NP trials [seed] [box].  Uses liblqro_hprof.so for fail reasons."""
import sys, os, ctypes as C, numpy as np
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "lqr-obstacles_amd"), os.path.join(ROOT, "oracle")]
import lqro, pyoracle as po
lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ.get("LQRO_LIB", "liblqro_hprof.so"))
L = lqro.lib()
N, H, NP, K = (int(a) for a in sys.argv[1:5])
kw = {}
if len(sys.argv) > 5: kw["seed"] = int(sys.argv[5])
if len(sys.argv) > 6: kw["box"] = float(sys.argv[6])
x, vg = lqro.synthetic_swarm(N, **kw)
g = lqro.synthesize_gains()
T, NCF = po.tables(g["A"], g["B"], g["L"], g["E"], H)
S = po.sphere(NP)
rv, rrecs = po.step(T, NCF, S, x, vg, threads=16)
inside = (rrecs["flags"] & 2) != 0
print("inside pairs", int(inside.sum()), flush=True)
c = lqro.Context(lqro.config(N, H, NP, flags=lqro.LQRO_FLAG_RECORDS))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
prev = np.zeros(32 + 2 * 4096 + 32, np.uint64)
bad_total = 0
for t in range(K):
    c.step(x, vg)
    recs = c.records()
    out = np.zeros_like(prev)
    L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
    d = out - prev
    prev = out
    fails = {k: int(d[16 + k]) for k in range(16) if d[16 + k]}
    bad = 0
    for r, q in zip(recs[inside], rrecs[inside]):
        if not (r["flags"] & 8) or not np.array_equal(r["facet"], q["facet"]) or r["dist"] != q["dist"]:
            bad += 1
            if bad <= 3:
                print("  mismatch pair", int(q["i"]), int(q["j"]), "flags", int(r["flags"]), r["facet"], q["facet"],
                      float(r["dist"]), float(q["dist"]), "n_facets", int(r["n_facets"]), int(q["n_facets"]))
    bad_total += bad
    print(f"trial {t}: ins {int(d[10])} conflicts {int(d[11])} stale {int(d[12])} fails {fails} bad {bad} "
          f"hull_ms {c.timings()['hull_ms']:.2f}", flush=True)
print("bad total", bad_total)
