"""Calibrate the reference-faithful CPU restatement (orc_step_faithful_mt)
against the reference's own pair loop compiled in this container
(oracle/_ref/libref.so ref_step, LQRO:1393-1436 with the reference's
functions): same rows of the C3 swarm, one thread each.  SURVEY §8d asks for
agreement within +-25 %.  Writes the result to the JSON path given."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "lqr-obstacles_amd")]
import pyoracle as o  # noqa: E402
import lqro  # noqa: E402

sys.path.insert(0, ROOT)
from bench import cpu_model  # noqa: E402

g = o.synthesize()
H, NP, N = 100, 100, 1024
x, vg = lqro.synthetic_swarm(N)
S = o.sphere(NP)
r = o.reflib()
assert r is not None, "needs oracle/_ref/libref.so (build container)"
r.ref_step.argtypes = [C.c_int] * 4 + [C.c_double] + [C.c_void_p] * 6 + [C.c_int, C.c_int, C.c_void_p, C.c_void_p]
p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
res = []
for rows in ((0, 4), (100, 104), (500, 504)):
    t0 = time.perf_counter()
    o.step_faithful(g["A"], g["B"], g["L"], g["E"], S, x, vg, H, rows=rows, records=False)
    tf = time.perf_counter() - t0
    nv = np.zeros((N, 3))
    ok = np.zeros(N, np.int32)
    t0 = time.perf_counter()
    r.ref_step(N, NP, H, 4, 30.0, p(g["A"]), p(g["B"]), p(g["L"]), p(g["E"]), p(np.ascontiguousarray(x)), p(vg),
               rows[0], rows[1], p(nv), p(ok))
    tr = time.perf_counter() - t0
    res.append({"rows": rows, "faithful_s": tf, "reference_s": tr, "ratio": tf / tr})
out = {"what": "orc_step_faithful_mt vs the reference's ref_step (libref.so), 1 thread, C3 rows",
       "cpu_model": cpu_model(), "runs": res,
       "ratio_mean": float(np.mean([q["ratio"] for q in res])),
       "pairs_per_s_faithful": 4 * (N - 1) * len(res) / sum(q["faithful_s"] for q in res),
       "pairs_per_s_reference": 4 * (N - 1) * len(res) / sum(q["reference_s"] for q in res)}
print(json.dumps(out, indent=1))
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        json.dump(out, f, indent=1)
