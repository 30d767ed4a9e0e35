"""Where the slowest Qhull-order builds spend their partitions: long
sequences (more than one 64-point chunk) against one-chunk ones, per build,
from a LQRO_QHULL_LONGPROF library (scripts/build_variant.sh liblqro_qlong.so
-DLQRO_QHULL_LONGPROF).  usage: LQRO_LIB=liblqro_qlong.so qhull_long.py [steps]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro  # noqa: E402
import numpy as np  # noqa: E402

if os.environ.get("LQRO_LIB"):
    lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ["LQRO_LIB"])
Q3_PROF_W1 = 32 + 2 * 4096 + 48 + 4 * 4096
Q3_PROF_LONG = Q3_PROF_W1 + 64
K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
for k in range(K):
    c.step(x, vg)
b = c.hull_builds()
w = np.zeros(24 * 1024, np.uint64)
fn = lqro.lib().lqro_debug_prof_words
fn.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]
assert fn(c._h, Q3_PROF_LONG, 24 * 1024, w.ctypes.data_as(C.c_void_p)) == 0
c.close()
w = w.reshape(-1, 24)[:len(b)]
d = (b["t_end"] - b["t_start"]) / 1e5
ok = b["kernel"] == 0
tot = d[ok].sum()
print(f"builds {ok.sum()}: {tot:.1f} ms; long-sequence insertions {w[ok, 0].sum() / ok.sum():.1f} per build, "
      f"{w[ok, 2].sum() / 1e5 / tot * 100:.1f} % of build time; all partitions {w[ok, 3].sum() / 1e5 / tot * 100:.1f} %")
print("wave 0 over all builds (% of build time): waiting for the speculation "
      f"{w[ok, 5].sum() / 1e5 / tot * 100:.1f}, adoption to publication {w[ok, 6].sum() / 1e5 / tot * 100:.1f}, "
      f"partitions {w[ok, 3].sum() / 1e5 / tot * 100:.1f} (long ones' locate {w[ok, 4].sum() / 1e5 / tot * 100:.1f}), "
      f"after the emit {w[ok, 7].sum() / 1e5 / tot * 100:.1f}")
print("slowest builds: ms, insertions, long insertions, long points, long ms (locate), all partitions ms, "
      "us/ins one-chunk; wave 0 ms: wait, adopt, tail")
for i in np.argsort(-d)[:8]:
    if not ok[i]:
        continue
    n_l, p_l, t_l, t_a, t_loc, t_w, t_ad, t_tl = (int(v) for v in w[i][:8])
    rest = d[i] - t_l / 1e5
    print(f"  {d[i]:7.2f} {b['insertions'][i]:5d} {n_l:4d} {p_l:6d} {t_l / 1e5:6.2f} ({t_loc / 1e5:5.2f}) {t_a / 1e5:6.2f} "
          f"{1e3 * rest / max(1, b['insertions'][i] - n_l):6.2f}; {t_w / 1e5:6.2f} {t_ad / 1e5:6.2f} {t_tl / 1e5:6.2f}")
    own, got, hw, hs, ev, po, hn, ht = (int(v) for v in w[i][8:16])
    print(f"      helped sequences: chunks wave 0 {own}, helpers {got}, waiting for helpers {hw / 1e5:.2f} ms, "
          f"stopping them {hs / 1e5:.2f} ms, events {ev}, posts {po}; helper chunks {hn}: "
          f"{(ht & 0xffffffff) / 1e2 / max(hn, 1):.2f} us locating, {(ht >> 32) / 1e2 / max(hn, 1):.2f} us claimed")
    ns, tps, tsd, tw0, nw0, nrl, tqs, thz = (int(v) for v in w[i][16:24])
    print(f"      wave 1: {ns} speculations, publication -> seen {tps / 1e2 / max(ns, 1):.2f} us, seen -> done "
          f"{tsd / 1e2 / max(ns, 1):.2f} us (queue scan {tqs / 1e2 / max(ns, 1):.2f}, {nrl} window reloads; horizon "
          f"{thz / 1e2 / max(ns, 1):.2f}); wave 0: {nw0} waits, speculation end -> seen {tw0 / 1e2 / max(nw0, 1):.2f} us")
