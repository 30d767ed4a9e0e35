"""The hull-bound regime: C3-sized swarms (1024 agents, H = 100) packed into
smaller boxes, so that more pairs end inside their LQR-obstacle hull.  Per
density: inside-hull pairs, step / sweep / LP time of the default (overlapped)
schedule, and the plain schedule's hull phase.  One process per schedule (a
second context would share hardware queues).
usage: crowded.py [--qhull] [side ...]   (default box sides 40 (the bench: 4 N^(1/3)), 30, 22, 16)
--qhull: the reference's hull rule (Qhull order, the library default) instead of the canonical one."""
import json, os, subprocess, sys
import numpy as np

if len(sys.argv) > 1 and sys.argv[1] == "--one":
    sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
    import lqro
    side = float(sys.argv[2])
    flags = lqro.LQRO_FLAG_QHULL_ORDER if os.environ.get("CROWDED_QHULL") == "1" else 0
    x, vg = lqro.synthetic_swarm(1024, box=side)
    g = lqro.synthesize_gains()
    c = lqro.Context(lqro.config(1024, 100, 100, flags=flags))
    c.set_gains(g["A"], g["B"], g["L"], g["E"])
    t = []
    for rnd in range(5):
        c.step(x, vg)
        if rnd >= 1:
            t.append(c.timings())
    st = c.stats()
    print(json.dumps({k: float(np.median([r[k] for r in t])) for k in ("step_ms", "pair_ms", "hull_ms", "lp_ms")}
                     | {"inside": int(st["inside"]), "hull_fail": int(st["hull_fail"])}))
    sys.exit(0)
rows = []
args = sys.argv[1:]
if args and args[0] == "--qhull":
    os.environ["CROWDED_QHULL"] = "1"
    args = args[1:]
for side in (args or ["40.3", "30", "22", "16"]):
    out = {"box_side_m": float(side)}
    for name, env in (("overlap", {"LQRO_HOT": "1"}), ("plain", {"LQRO_HOT": "0"})):
        r = subprocess.run([sys.executable, __file__, "--one", side], env={**os.environ, **env},
                           capture_output=True, text=True, timeout=300)
        out[name] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-300:]
    rows.append(out)
    print(json.dumps(out), flush=True)
