"""A pair whose hull the in-kernel hulls cannot build is reported, never
dropped silently: the reference always gets a hull from qconvex
(LQRObstacles.cpp:879-880), so a missing half-plane is an error of this
build.  liblqro_tinycap.so (__graft_entry__.build_tinycap_lib) is liblqro.so
with k_qhull's and k_qhull_big's per-insertion caps cut to 4 visible / 8 new
facets: on a dense swarm in the default rule (Qhull order) most hulls exceed
them.  lqro_step must then return LQRO_E_HULL (lqro.HullFailure), name the
pairs (lqro_get_hull_failures), count them (stats hull_fail) and mark their
records; every other pair's record must equal the full library's.  One step:
the capped builds go to k_qhull_big through the retry queue; the third step
(builds were capped two steps before): k_qhull<true> rebuilds them in place
(q3_big_inline) — the same failures, the same records."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

PKG = os.path.join(ROOT, "lqr-obstacles_amd")
SWARM = dict(n=24, box=3.0, seed=11, H=45)

CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import lqro
lqro.LIB_PATH = sys.argv[2]
a = json.loads(sys.argv[3])
x, vg = lqro.synthetic_swarm(a["n"], box=a["box"], seed=a["seed"])
g = lqro.synthesize_gains()
c = lqro.Context(lqro.config(a["n"], a["H"], 100, flags=lqro.LQRO_FLAG_RECORDS | lqro.LQRO_FLAG_QHULL_ORDER))
c.set_gains(g["A"], g["B"], g["L"], g["E"])
for t in range(a["steps"]):
    out = {"raised": False, "pairs": []}
    try:
        c.step(x, vg)
    except lqro.HullFailure as e:
        out["raised"] = True
        out["pairs"] = [[int(i), int(j)] for i, j in e.pairs]
r = c.records()
st = c.stats()
out["hull_fail"] = st["hull_fail"]
out["fail_ij"] = [[int(q["i"]), int(q["j"])] for q in r[(r["flags"] & lqro.REC_HULLFAIL) != 0]]
np.save(sys.argv[4], r)
print(json.dumps(out))
"""


@pytest.mark.parametrize("steps", [1, 3])
def test_capacity_failures_are_reported(lqro_mod, tmp_path, steps):
    lib = os.path.join(PKG, "liblqro_tinycap.so")
    assert os.path.exists(lib), "liblqro_tinycap.so not built (__graft_entry__.build)"
    rp = str(tmp_path / "recs.npy")
    res = subprocess.run([sys.executable, "-c", CHILD, PKG, lib, json.dumps(dict(SWARM, steps=steps)), rp],
                         capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    small = np.load(rp)
    # the full library: every inside pair gets its plane
    x, vg = lqro_mod.synthetic_swarm(SWARM["n"], box=SWARM["box"], seed=SWARM["seed"])
    g = lqro_mod.synthesize_gains()
    c = lqro_mod.Context(lqro_mod.config(SWARM["n"], SWARM["H"], 100,
                                         flags=lqro_mod.LQRO_FLAG_RECORDS | lqro_mod.LQRO_FLAG_QHULL_ORDER))
    c.set_gains(g["A"], g["B"], g["L"], g["E"])
    c.step(x, vg)
    full = c.records()
    assert c.stats()["hull_fail"] == 0
    c.close()
    inside = (full["flags"] & lqro_mod.REC_INSIDE) != 0
    assert inside.sum() > 4
    # the failures: raised, counted, named, marked
    assert out["raised"], "lqro_step returned OK with hulls it could not build"
    nf = out["hull_fail"]
    assert nf > 0 and nf == len(out["fail_ij"])
    # lqro_get_hull_failures names the first min(nf, 64) failures in completion
    # order, not the smallest (i, j): every named pair is a failed one
    named = set(map(tuple, out["pairs"]))
    assert len(out["pairs"]) == min(nf, 64) and len(named) == len(out["pairs"])
    assert named <= set(map(tuple, out["fail_ij"]))
    failed = (small["flags"] & lqro_mod.REC_HULLFAIL) != 0
    assert np.all(inside[failed])
    # every pair the caps did not touch is the full library's, bit for bit
    ok = ~failed
    ok &= ~inside | ((small["flags"] & lqro_mod.REC_STALE) == 0)   # (a stale normal may come from a failed pair)
    for f in ("n_reach", "reach_hash", "facet", "dist"):
        assert np.array_equal(small[f][ok], full[f][ok]), f
