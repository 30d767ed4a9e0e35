#!/usr/bin/env python3
"""C3 in Qhull order: when each build starts relative to the step's first hot
pair, and how long after its own pair's evaluation ended (needs liblqro_hs.so:
scripts/build_variant.sh liblqro_hs.so -DLQRO_HOT_STAMPS).  All times on the
100 MHz clock (hot stamps and lqro_get_hull_builds share it).
usage: LQRO_LIB=liblqro_hs.so python3 scripts/hot_build_timeline.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import lqro  # noqa: E402

lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ.get("LQRO_LIB", "liblqro_hs.so"))
L = lqro.lib()
N, H, NP = 1024, 100, 100
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(N, H, NP, flags=lqro.LQRO_FLAG_QHULL_ORDER))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
off = 32 + 2 * 4096 + 48
for k in range(6):
    c.step(x, vg)
    tm = c.timings()
    w = np.zeros(2 * 8192, np.uint64)
    L.lqro_debug_prof_words(c._h, C.c_int64(off), C.c_int64(2 * 8192), w.ctypes.data_as(C.c_void_p))
    st = w[0::2].astype(np.int64)
    en = (w[1::2] & np.uint64((1 << 63) - 1)).astype(np.int64)
    ok = st > 0
    t0 = st[ok].min()
    b = c.hull_builds()
    done = b[b["kernel"] != 2]
    bs = (done["t_start"].astype(np.int64) - t0) / 100.0
    be = (done["t_end"].astype(np.int64) - t0) / 100.0
    k_slow = int(np.argmax(be - bs))
    print(f"step {k}: device {tm['pair_ms'] + tm['hull_ms'] + tm['lp_ms']:.2f} ms; {ok.sum()} hot pairs, last hot end "
          f"{(en[ok].max() - t0) / 100:.0f} us; builds {len(done)}: start min {bs.min():.0f} p50 {np.median(bs):.0f} "
          f"max {bs.max():.0f} us, last end {be.max() / 1000:.3f} ms; slowest ({int(done['i'][k_slow])}, "
          f"{int(done['j'][k_slow])}) starts {bs[k_slow]:.0f} us, ends {be[k_slow] / 1000:.3f} ms", flush=True)
    w[:] = 0
c.close()
