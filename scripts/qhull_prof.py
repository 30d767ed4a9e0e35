"""k_qhull phase profile of one C3 step in Qhull order (needs
liblqro_qprof.so: scripts/build_variant.sh liblqro_qprof.so -DLQRO_QHULL_PROFILE):
cycles per phase summed over the step's hulls (s_memtime, 100 MHz)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro  # noqa: E402

lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ.get("LQRO_LIB", "liblqro_qprof.so"))
L = lqro.lib()
box = float(sys.argv[1]) if len(sys.argv) > 1 else None
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N, box=box) if box else lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP, flags=lqro.LQRO_FLAG_QHULL_ORDER))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
c.step(x, vg)
print(c.timings(), c.stats())
out = np.zeros(32 + 2 * 4096 + 32, np.uint64)
L.lqro_debug_hull_profile(c._h, out.ctypes.data_as(C.c_void_p))
names = ["init+partitionall", "nextfurthest", "findhorizon", "makenew", "match+planes+checkzero",
         "gather", "locate", "emit", "delvertex", "delete+reset", "select", "jobs",
         "locate:fetch", "locate:search", "locate:count", "emit:segments", "emit:loads", "emit:groups",
         "emit:final+queue", "makenew:ridges", "sharp", "-", "-", "-"]
jobs = max(int(out[11]), 1)
ks = [k for k in range(24) if k != 11 and names[k] != "-"]
tot = sum(int(out[k]) for k in ks)
GHZ = 2.4   # s_memtime counts shader cycles (MI355X_MICROARCH.md, PMC units)
for k in ks:
    print(f"{names[k]:24s} {int(out[k]) / jobs / GHZ / 1e6:10.3f} ms/hull  {100 * int(out[k]) / max(tot, 1):5.1f}%")
print("hulls", jobs, "phase sum ms/hull", tot / jobs / GHZ / 1e6)
print("job ms/hull (mean, max)", int(out[27]) / jobs / GHZ / 1e6, int(out[26]) / GHZ / 1e6,
      "points/hull", int(out[28]) / jobs)
for k, nm in ((21, "insertions"), (22, "partitioned points"), (23, "located chunks"), (24, "sequence events"),
              (25, "emitted groups")):
    print(f"{nm:24s} {int(out[k]) / jobs:12.1f} per hull")
print("insertions adopted from wave 1's speculation:", int(out[31]) / jobs, "per hull")
print("insertions with > 64 partitioned points:", int(out[30]) / jobs, "per hull,",
      int(out[29]) / jobs / GHZ / 1e6, "ms per hull")
nj = min(jobs, 4096)
pj = out[32:32 + 2 * nj].reshape(nj, 2)
cyc = pj[:, 0].astype(np.float64) / GHZ / 1e6
ins = (pj[:, 1] & 0xFFFFF).astype(np.int64)
npt = ((pj[:, 1] >> 20) & 0xFFFFF).astype(np.int64)
nsl = (pj[:, 1] >> 40).astype(np.int64)
o = np.argsort(-cyc)
print("slowest hulls: ms, insertions, points, facet slots, us/insertion")
for k in o[:8]:
    print(f"  {cyc[k]:8.3f} {ins[k]:6d} {npt[k]:6d} {nsl[k]:6d} {1e3 * cyc[k] / max(ins[k], 1):8.2f}")
print("us/insertion: all", 1e3 * cyc.sum() / max(ins.sum(), 1),
      "slots < 2752:", 1e3 * cyc[nsl < 2752].sum() / max(ins[nsl < 2752].sum(), 1),
      "slots >= 2752:", 1e3 * cyc[nsl >= 2752].sum() / max(ins[nsl >= 2752].sum(), 1), int((nsl >= 2752).sum()), "hulls")
nr = int(out[32 + 2 * 4096 + 16])
if nr:
    caps = {0x100: "horizon walk", 0x200: "coplanar set", 0x400: "moved facets", 0x800: "outside-set buffer",
            0x1000: "visible facets", 0x2000: "new facets", 0x4000: "facet slots / queue"}
    st = int(out[32 + 2 * 4096 + 17])
    print("builds handed to k_qhull_big:", nr, "caps:", [v for b, v in caps.items() if st & b],
          "slots:", [(int(w) & 0xffffffff, hex(int(w) >> 32)) for w in out[32 + 2 * 4096 + 18:32 + 2 * 4096 + 18 + min(nr, 14)]])

W1 = 32 + 2 * 4096 + 48 + 4 * 4096   # Q3_PROF_W1
wv = np.zeros(64, np.uint64)
L.lqro_debug_prof_words(c._h, C.c_int64(W1), C.c_int64(64), wv.ctypes.data_as(C.c_void_p))
w1 = [int(v) for v in wv]
if w1[7]:
    print("wave 1: speculations", w1[7] / jobs, "per hull,", w1[0] / max(w1[7], 1) / GHZ / 1e3, "us each;",
          "phases us/spec: records %.2f queue %.2f horizon %.2f cone %.2f match %.2f checkzero %.2f sharp %.2f;"
          " horizon levels %.2f" %
          (tuple(w1[k] / max(w1[7], 1) / GHZ / 1e3 for k in (1, 2, 3, 4, 12, 13, 5)) + (w1[11] / max(w1[7], 1),)))
    print("handshake: publication -> speculation start %.3f us, speculation end -> wave 0 sees it %.3f ms/hull"
          " (when it waited); waits after one-chunk insertions %.3f us each (%d)" %
          (w1[14] / max(w1[7], 1) / GHZ / 1e3, w1[41] / jobs / GHZ / 1e6, w1[42] / max(w1[43], 1) / GHZ / 1e3,
           w1[43] // jobs))
    print("after one-chunk insertions: publication -> speculation end %.3f us, -> wave 0 past its wait %.3f us" %
          (w1[44] / max(w1[43], 1) / GHZ / 1e3, w1[45] / max(w1[43], 1) / GHZ / 1e3))
    print("  the wait's first read back %.3f us, spins %.2f; publication -> after wave 1's store %.3f us" %
          (w1[46] / max(w1[43], 1) / GHZ / 1e3, w1[47] / max(w1[43], 1), w1[48] / max(w1[43], 1) / GHZ / 1e3))
    print("  wave 0's publication release %.3f us each (all insertions)" % (w1[49] / max(w1[10], 1) / GHZ / 1e3))
    print("  real-time clock (100 MHz), after one-chunk insertions: publication -> spec start %.3f us, -> spec end %.3f us,"
          " -> wave 0 sees it %.3f us (global copy %.3f)" % tuple(w1[k] / max(w1[43], 1) / 100.0 for k in (50, 51, 52, 53)))
    print("  each wave's own clock: wave 1 idle between speculations %.3f us; wave 0 from seeing one to the next publication %.3f us"
          % (w1[15] / max(w1[7], 1) / GHZ / 1e3, w1[54] / max(w1[55], 1) / GHZ / 1e3))
    print("  (STARTSIG builds) wave 0 sees wave 1 start %.3f us after publishing" % (w1[56] / max(w1[55], 1) / GHZ / 1e3))
    print("wave 1: chunks served", w1[8] / jobs, "per hull,", w1[6] / max(w1[8], 1) / GHZ / 1e3, "us each")
    print("wave 0 waiting for a speculation: %.3f ms/hull, %.2f us per wait (%d waits/hull)" %
          (w1[9] / jobs / GHZ / 1e6, w1[9] / max(w1[10], 1) / GHZ / 1e3, w1[10] // jobs))
nps = w1[16 + 24]
if nps:
    print("one-chunk insertions (np <= 64): %.1f per hull; us per insertion by phase:" % (nps / jobs))
    tot1 = 0
    for k in range(21):
        if k != 11 and names[k] != "-":
            v = w1[16 + k] / nps / GHZ / 1e3
            tot1 += v
            print(f"    {names[k]:24s} {v:8.3f}")
    print("    total %.3f us" % tot1)
