"""When the hot launch's pairs end (needs liblqro_hs.so: scripts/build_variant.sh
liblqro_hs.so -DLQRO_HOT_STAMPS): per C3 step, the 100 MHz start / end of each
hot pair relative to the launch's first start, for the inside-hull pairs and
for all.  usage: LQRO_LIB=liblqro_hs.so python3 scripts/hot_stamps.py"""
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
c = lqro.Context(lqro.config(N, H, NP))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
off = 32 + 2 * 4096 + 48
for k in range(5):
    c.step(x, vg)
    w = np.zeros(2 * 8192, np.uint64)
    L.lqro_debug_prof_words(c._h, C.c_int64(off), C.c_int64(2 * 8192), w.ctypes.data_as(C.c_void_p))
    st = w[0::2].astype(np.int64)
    en_raw = w[1::2]
    ok = st > 0
    ins = ((en_raw >> np.uint64(63)) & np.uint64(1)).astype(bool) & ok
    en = (en_raw & np.uint64((1 << 63) - 1)).astype(np.int64)
    t0 = st[ok].min()
    e_all = (en[ok] - t0) / 100.0  # us
    e_in = (en[ins] - t0) / 100.0
    d_all = (en[ok] - st[ok]) / 100.0
    d_in = (en[ins] - st[ins]) / 100.0
    print(f"step {k}: {ok.sum()} hot pairs, {ins.sum()} inside; end of all: max {e_all.max():.0f} us, "
          f"p50 {np.percentile(e_all, 50):.0f}, p90 {np.percentile(e_all, 90):.0f}; inside ends: "
          f"max {e_in.max() if ins.any() else 0:.0f} us, p50 {np.percentile(e_in, 50) if ins.any() else 0:.0f}; "
          f"pair time inside mean {d_in.mean() if ins.any() else 0:.0f} max {d_in.max() if ins.any() else 0:.0f} us, "
          f"non-inside mean {d_all[~ins[ok]].mean():.0f} max {d_all[~ins[ok]].max():.0f} us", flush=True)
    w[:] = 0
