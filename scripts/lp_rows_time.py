"""Run lqro_calculate_new_v on the C3 swarm's hardest LP rows
(tests/golden/lp_rows.npz) a few times and check them bit for bit; under
rocprofv3 --kernel-trace --stats the k_lp4 line is linearProgram4's latency
(one workgroup a row, all rows at once)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lqr-obstacles_amd")]
import lqro  # noqa: E402

if os.environ.get("LQRO_LIB"):
    lqro.LIB_PATH = os.path.join(os.path.dirname(lqro.LIB_PATH), os.environ["LQRO_LIB"])
d = np.load(os.path.join(ROOT, "tests", "golden", "lp_rows.npz"))
rows = int(sys.argv[1]) if len(sys.argv) > 1 else len(d["newv"])
for it in range(5):
    got = lqro.calculate_new_v(list(d["planes"][:rows]), d["vgoal"][:rows], vmax_lp=float(d["vmax_lp"]))
    ok = np.array_equal(got.view(np.uint64), d["newv"][:rows].view(np.uint64))
    print("iter", it, "bit-exact" if ok else "MISMATCH", flush=True)
    if not ok:
        sys.exit(1)
