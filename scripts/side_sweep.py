"""C3 step time across side-stream widths (LQRO_SIDE_HULL_CUS) and the plain
schedule (LQRO_HOT=0).  One process per setting: a second context in a process
shares hardware queues and serialises the overlap.
usage: side_sweep.py [widths...]     (child: side_sweep.py --one)"""
import os, subprocess, sys
import numpy as np

if len(sys.argv) > 1 and sys.argv[1] == "--one":
    sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
    import lqro
    if os.environ.get("LQRO_LIB"):   # a variant build (lqr-obstacles_amd/<name>)
        lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ["LQRO_LIB"])
    N, H, NP = 1024, 100, 100
    x, vg = lqro.synthetic_swarm(N)
    g = lqro.synthesize_gains()
    c = lqro.Context(lqro.config(N, H, NP, flags=0))
    c.set_gains(g["A"], g["B"], g["L"], g["E"])
    t = []
    for rnd in range(8):
        c.step(x, vg)
        if rnd >= 2:
            t.append(c.timings())
    print("step_ms %.2f pair_ms %.2f hull_ms %.2f lp_ms %.2f" % tuple(
        np.median([r[k] for r in t]) for k in ("step_ms", "pair_ms", "hull_ms", "lp_ms")))
    sys.exit(0)
settings = [("plain", {"LQRO_HOT": "0"})] + [(f"side{w}", {"LQRO_HOT": "1", "LQRO_SIDE_HULL_CUS": w})
                                             for w in (sys.argv[1:] or ["48", "64", "96", "128"])]
for name, env in settings:
    r = subprocess.run([sys.executable, __file__, "--one"], env={**os.environ, **env}, capture_output=True,
                       text=True, timeout=120)
    print(name, r.stdout.strip() or r.stderr[-400:], flush=True)
